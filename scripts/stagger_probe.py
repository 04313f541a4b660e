"""Probe: does the relative placement of the DiLoCo step's 10 streams (8 fp32 workers, theta,
momentum) set its rate? bench.py's momentum placement by measurement (placement.py) sees up to
11 % between allocations of the same buffer. Here the K + 2 arenas are carved out of ONE
allocation at base offsets k x (P x 4 + D) for a stagger D, so the streams' relative offsets
are controlled; each layout is timed with the real fused step (edt_outer_step) and the
access-pattern probe (edt_probe_stream), HIP events, median of `--iters`.

    python scripts/stagger_probe.py [--staggers 0,256,4096,65536,1048576,2101248]
"""
from __future__ import annotations

import argparse
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def _median_ms(fn, iters):
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
    from evolutionarydistributedtraining_amd import _lib as L
    from evolutionarydistributedtraining_amd import ops
    from evolutionarydistributedtraining_amd.layouts import gpt_1p3b
    ap = argparse.ArgumentParser()
    ap.add_argument("--staggers", default="0,256,4096,65536,1048576,2101248")
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--k", type=int, default=8)
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    P, K = gpt_1p3b().total, a.k
    nbytes = P * 4
    algo = (K * 4 + 16) * P
    lib = L.lib()
    st = L.stream_ptr(dev)
    res = {"P": P, "K": K, "algo_bytes": algo, "layouts": []}

    def run_layout(name, arenas):
        theta, mom, workers = arenas[0], arenas[1], arenas[2:]
        g = torch.Generator(device=dev).manual_seed(1)
        theta.copy_(torch.randn(P, device=dev, generator=g) * 0.02)
        for w in workers:
            w.copy_(theta)
        mom.zero_()
        arr = L.ptr_array(workers)
        step = lambda: ops.outer_step(theta, workers, mom, True, 0.7, 0.9, True)
        probe = lambda: L.check(lib.edt_probe_stream(L.ptr(theta), 0, arr, 0, K, L.ptr(mom), P, st), "probe")
        ms = [_median_ms(step, a.iters), _median_ms(probe, a.iters)]
        row = {"layout": name, "step_ms": round(ms[0], 3), "probe_ms": round(ms[1], 3),
               "step_frac": round(algo / (ms[0] / 1e3) / 1e9 / 8000, 4),
               "base_mod_2MiB": [int(t.data_ptr() % (2 << 20)) for t in arenas[:3]]}
        res["layouts"].append(row)
        print(json.dumps(row), file=sys.stderr, flush=True)

    # separate allocations (what the bench does before placement), twice
    for rep in range(2):
        arenas = [torch.empty(P, device=dev) for _ in range(K + 2)]
        run_layout(f"separate_{rep}", arenas)
        del arenas
        torch.cuda.empty_cache()
    for d in [int(x) for x in a.staggers.split(",")]:
        stride = (nbytes + d + 255) // 256 * 256
        pool = torch.empty(stride * (K + 2) + 256, dtype=torch.uint8, device=dev)
        base = (-pool.data_ptr()) % 256
        arenas = [pool[base + k * stride: base + k * stride + nbytes].view(torch.float32) for k in range(K + 2)]
        run_layout(f"stagger_{d}", arenas)
        del arenas, pool
        torch.cuda.empty_cache()
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
