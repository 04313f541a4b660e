"""Does the fused step's speed depend on where momentum sits relative to theta? theta and the
momentum are the step's two read-modify-write streams. This carves both out of ONE allocation,
with the momentum starting `gap` bytes after the end of theta, sweeps the gap, and times the
product kernel on each placement. The 8 fp32 workers stay in their own allocations throughout.
Prints one JSON object.

    python scripts/mom_offset_sweep.py [--step-mib 256] [--count 24]
"""
from __future__ import annotations

import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from scripts.alloc_draws import time_step  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--params", type=int, default=1315723264)
    ap.add_argument("--workers", type=int, default=8)
    ap.add_argument("--step-mib", type=int, default=256)
    ap.add_argument("--count", type=int, default=24)
    ap.add_argument("--small", default="0,2,4,8,16,32,64,128",
                    help="extra gaps in MiB below one step (low-address-bit staggers)")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    n, k = a.params, a.workers
    step = a.step_mib * (1 << 20) // 4
    gaps = sorted({int(x) * (1 << 20) // 4 for x in a.small.split(",")} | {j * step for j in range(a.count)})
    big = torch.empty(2 * n + max(gaps), device=dev)
    theta0 = torch.randn(n, device=dev) * 0.02
    mom0 = torch.randn(n, device=dev) * 1e-4
    workers = []
    for _ in range(k):
        w = torch.empty(n, device=dev)
        w.copy_(theta0)
        workers.append(w)
    # reference: theta and momentum in allocations of their own (the bench's arrangement)
    res = {"params": n, "separate_allocations_ms": None, "gap_MiB_to_ms": {}}
    res["separate_allocations_ms"] = round(time_step(theta0.clone(), workers, mom0.clone()), 4)
    for gap in gaps:
        theta = big[:n]
        mom = big[n + gap:2 * n + gap]
        theta.copy_(theta0)
        mom.copy_(mom0)
        ms = time_step(theta, workers, mom)
        res["gap_MiB_to_ms"][f"{gap * 4 / (1 << 20):g}"] = round(ms, 4)
        print(f"gap {gap * 4 / (1 << 20):8g} MiB  {ms:.4f} ms", flush=True)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
