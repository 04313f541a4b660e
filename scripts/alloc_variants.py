"""Do build variants of the fused outer step change how much the momentum's PLACEMENT costs?

The step's speed depends on where the momentum sits physically relative to theta (placement.py,
DESIGN §6.0): the same launch takes ~10.5 ms on good placements and ~11.5 on bad ones. This probe
makes one theta + 8 fp32 workers (bench.py's 1.3B configuration) and several momentum buffers
spread by held spacers (as placement.place_momentum does), then times every variant library (built
by scripts/kernel_variants.py --build) on every momentum buffer, interleaved. A variant that makes
the bad placements as fast as the good ones would remove the need for the search.

    python scripts/kernel_variants.py --build --variants default,f32_ntst,nt_rmw_st,xcd_full,f32_bpc64   # here
    python scripts/alloc_variants.py --variants default,f32_ntst,nt_rmw_st,xcd_full,f32_bpc64            # GPU box
"""
import argparse
import ctypes
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from kernel_variants import VDIR  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--variants", default="default,f32_ntst,nt_rmw_st,xcd_full,f32_bpc64")
    ap.add_argument("--placements", type=int, default=6)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--iters", type=int, default=5)
    a = ap.parse_args()
    from evolutionarydistributedtraining_amd import _lib as L
    from evolutionarydistributedtraining_amd.layouts import gpt_1p3b
    dev = torch.device("cuda:0")
    P = gpt_1p3b().total
    # (theta, momentum) pairs: the momentum right after theta (the first allocation's usual case),
    # both carved from ONE allocation (a flat ~11.6 ms at any gap), and momentum
    # buffers spread by held spacers
    theta = torch.randn(P, device=dev) * 0.02
    adjacent = torch.zeros(P, device=dev)
    workers = [theta + torch.randn(P, device=dev) * 1e-3 for _ in range(8)]
    carved = torch.zeros(2 * P, device=dev)
    carved[:P].copy_(theta)
    pairs = [("adjacent", theta, adjacent), ("carved", carved[:P], carved[P:])]
    spacers = []
    for c in range(1, a.placements):
        spacers.append(torch.empty(c * (11 << 27), dtype=torch.uint8, device=dev))
        pairs.append((f"spread{c}", theta, torch.zeros(P, device=dev)))
    names = a.variants.split(",")
    libs = {}
    for n in names:
        f = ctypes.CDLL(os.path.join(VDIR, f"{n}.so")).edt_outer_step
        f.restype = ctypes.c_int
        f.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.POINTER(ctypes.c_void_p), ctypes.c_int, ctypes.c_int,
                      ctypes.c_void_p, ctypes.c_int, ctypes.c_uint64, ctypes.c_double, ctypes.c_double,
                      ctypes.c_int, ctypes.c_void_p]
        libs[n] = f
    arr = L.ptr_array(workers)
    st = L.stream_ptr(dev)

    def launch(f, th, m):
        assert f(ctypes.c_void_p(th.data_ptr()), 0, arr, 0, 8, ctypes.c_void_p(m.data_ptr()), 1, P, 0.7, 0.9, 1,
                 st) == 0
    for n in names:
        for _, th, m in pairs:
            launch(libs[n], th, m)
    torch.cuda.synchronize()
    times = {(n, j): [] for n in names for j in range(len(pairs))}
    for _ in range(a.rounds):
        for j, (_, th, m) in enumerate(pairs):
            for n in names:
                evs = [torch.cuda.Event(enable_timing=True) for _ in range(2 * a.iters)]
                for i in range(a.iters):
                    evs[2 * i].record()
                    launch(libs[n], th, m)
                    evs[2 * i + 1].record()
                torch.cuda.synchronize()
                times[(n, j)] += [evs[2 * i].elapsed_time(evs[2 * i + 1]) for i in range(a.iters)]
        print("round done", file=sys.stderr, flush=True)
    res = {n: {pairs[j][0]: round(statistics.median(times[(n, j)]), 4) for j in range(len(pairs))} for n in names}
    print(json.dumps({"probe": "alloc_variants", "P": P, "K": 8, "dtype": "f32",
                      "momentum_minus_theta_GiB": {nm: round((m.data_ptr() - th.data_ptr()) / 2**30, 3)
                                                   for nm, th, m in pairs},
                      "median_ms_by_placement": res}, indent=1))


if __name__ == "__main__":
    main()
