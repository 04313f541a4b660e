"""Probe: is a joint placement search over theta AND the momentum worth more than the momentum
alone (placement.place_momentum, what bench.py does)? The 1.3B fp32 x 8 step's access pattern
(edt_probe_stream) is timed for every (theta candidate, momentum candidate) pair, candidates being
fresh allocations spread by spacer allocations as place_momentum spreads them; reports the
momentum-only best (theta = its first allocation), the joint best, and the full grid.

    python scripts/joint_placement_probe.py [--theta 4 --mom 8]
"""
from __future__ import annotations

import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from evolutionarydistributedtraining_amd import placement
    from evolutionarydistributedtraining_amd.layouts import gpt_1p3b
    ap = argparse.ArgumentParser()
    ap.add_argument("--theta", type=int, default=4)
    ap.add_argument("--mom", type=int, default=8)
    ap.add_argument("--spacer", type=int, default=11 << 27)
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    P = gpt_1p3b().total
    workers = [torch.zeros(P, device=dev) for _ in range(8)]
    keep = []
    thetas, moms = [], []
    for c in range(a.theta):
        if c:
            keep.append(torch.empty(c * a.spacer, dtype=torch.uint8, device=dev))
        thetas.append(torch.zeros(P, device=dev))
    for c in range(a.mom):
        if c:
            keep.append(torch.empty(c * a.spacer, dtype=torch.uint8, device=dev))
        moms.append(torch.zeros(P, device=dev))
    grid = [[round(placement.probe_ms(th, workers, m, iters=3), 4) for m in moms] for th in thetas]
    mom_only = min(grid[0])
    joint = min(min(r) for r in grid)
    res = {"P": P, "grid_ms": grid, "momentum_only_best_ms": mom_only, "joint_best_ms": joint,
           "gain": round(mom_only / joint - 1, 4)}
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
