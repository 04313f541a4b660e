"""Probe: what rate does the two-pass SLERP (and a plain lerp) reach when its working set fits the
256 MiB Infinity Cache and is re-run back to back (the data stays on-die between runs), against
working sets far larger than it? If on-die re-reads stream much faster than HBM, a per-tensor
fused stats -> blend schedule could hide the second read of the parents.

    python scripts/mall_rate_probe.py [--elems 4194304,8388608,16777216,33554432,67108864,268435456]
"""
from __future__ import annotations

import argparse
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def _ms(fn, iters=20):
    fn()
    torch.cuda.synchronize()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(iters)]
    for a, b in ev:
        a.record()
        fn()
        b.record()
    torch.cuda.synchronize()
    return statistics.median(a.elapsed_time(b) for a, b in ev)


def main():
    from evolutionarydistributedtraining_amd import ops
    ap = argparse.ArgumentParser()
    ap.add_argument("--elems", default="4194304,8388608,16777216,33554432,67108864,268435456")
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    bf = torch.bfloat16
    rows = []
    for n in [int(x) for x in a.elems.split(",")]:
        g = torch.Generator(device=dev).manual_seed(1)
        v0 = (torch.randn(n, generator=g, device=dev) * 0.02).to(bf)
        v1 = (v0.float() + torch.randn(n, generator=g, device=dev) * 0.02).to(bf)   # far: SLERP branch
        out = torch.empty(n, dtype=bf, device=dev)
        plan = ops.make_slerp_plan([0, n], dev)
        t = torch.full((1,), 0.5, dtype=torch.float64, device=dev)
        two = _ms(lambda: ops.slerp_arena(plan, v0, v1, out, t, speculate=False))
        lerp = _ms(lambda: ops.lerp(0.5, v0, v1, out))
        row = {"elems": n, "parents_MiB": 4 * n / 2**20,
               "two_pass_ms": round(two, 4), "two_pass_moved_TBps": round(10 * n / (two / 1e3) / 1e12, 2),
               "lerp_ms": round(lerp, 4), "lerp_TBps": round(6 * n / (lerp / 1e3) / 1e12, 2)}
        rows.append(row)
        print(json.dumps(row), file=sys.stderr, flush=True)
        del v0, v1, out, plan
        torch.cuda.empty_cache()
    print(json.dumps(rows), flush=True)


if __name__ == "__main__":
    main()
