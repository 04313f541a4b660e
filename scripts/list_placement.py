"""Does the momentum's placement matter for the tensor-list outer step too? The base model's
parameters and the workers are separate allocations per tensor (gpt_1p3b: 292 per model, as
models loaded straight to the GPU), the momentum one flat buffer viewed per tensor (OuterState).
Times ops.outer_step_list with the momentum in C spaced candidate allocations (the spacers of
placement.place_momentum) and with the momentum as separate per-tensor allocations.

    python scripts/list_placement.py [--wdt bf16] [--candidates 6]
"""
from __future__ import annotations

import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from evolutionarydistributedtraining_amd import ops  # noqa: E402
from evolutionarydistributedtraining_amd.layouts import gpt_1p3b  # noqa: E402


def timed(fn, iters=7):
    fn()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(iters)]
    for a, b in ev:
        a.record()
        fn()
        b.record()
    torch.cuda.synchronize()
    ts = sorted(a.elapsed_time(b) for a, b in ev)
    return ts[len(ts) // 2]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--wdt", default="bf16", choices=["bf16", "f32"])
    ap.add_argument("--candidates", type=int, default=6)
    ap.add_argument("--spacer-bytes", type=int, default=11 << 27)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    lay = gpt_1p3b()
    wdt = torch.bfloat16 if a.wdt == "bf16" else torch.float32
    thetas = [torch.randn(s, device=dev) * 0.02 for s in lay.shapes]
    workers = [[(t + torch.randn_like(t) * 1e-3).to(wdt) for t in thetas] for _ in range(8)]
    res = {"wdt": a.wdt, "flat_momentum_candidates_ms": [], "per_tensor_momentum_ms": None}
    keep = []
    for c in range(a.candidates):
        if c:
            keep.append(torch.empty(c * a.spacer_bytes, dtype=torch.uint8, device=dev))
        mom = torch.zeros(lay.total, device=dev)
        keep.append(mom)
        views = lay.views(mom)
        ms = timed(lambda: ops.outer_step_list(thetas, workers, views, True, 0.7, 0.9, True))
        res["flat_momentum_candidates_ms"].append(round(ms, 4))
        print("candidate", c, round(ms, 4), flush=True)
    del keep
    moms = [torch.zeros_like(t) for t in thetas]
    res["per_tensor_momentum_ms"] = round(timed(lambda: ops.outer_step_list(thetas, workers, moms, True, 0.7, 0.9,
                                                                            True)), 4)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
