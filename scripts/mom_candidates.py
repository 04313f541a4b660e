"""How often does a fresh allocation give the momentum a fast placement? Allocates theta and 8
fp32 workers (separate allocations, as the bench does), then a sequence of momentum candidates,
each preceded by a spacer allocation of a chosen size (shifting where the candidate lands), and
times the step's access pattern (edt_probe_stream) on every candidate. Prints one JSON object.

    python scripts/mom_candidates.py [--spacers-mib 0,2,32,256,1024,2560,0,0,4096,128]
"""
from __future__ import annotations

import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from evolutionarydistributedtraining_amd.placement import probe_ms  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--params", type=int, default=1315723264)
    ap.add_argument("--workers", type=int, default=8)
    ap.add_argument("--spacers-mib", default="0,2,32,256,1024,2560,0,0,4096,128,0,512")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    n = a.params
    theta = torch.randn(n, device=dev) * 0.02
    workers = [theta.clone() for _ in range(a.workers)]
    keep, res = [], []
    for sp in (int(x) for x in a.spacers_mib.split(",")):
        if sp:
            keep.append(torch.empty(sp * (1 << 20), dtype=torch.uint8, device=dev))
        mom = torch.zeros(n, device=dev)
        keep.append(mom)
        ms = probe_ms(theta, workers, mom, iters=5)
        res.append({"spacer_MiB": sp, "probe_ms": round(ms, 4), "offset_GiB": round((mom.data_ptr() - theta.data_ptr()) / 2**30, 3)})
        print(json.dumps(res[-1]), flush=True)
    # the same candidates again, in reverse order: is each placement's speed stable?
    again = [round(probe_ms(theta, workers, m, iters=5), 4) for m in keep if m.numel() == n][::-1]
    print(json.dumps({"candidates": res, "again_reversed": again}))


if __name__ == "__main__":
    main()
