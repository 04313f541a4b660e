"""Probe: does the fused step's time depend on the RELATIVE placement of its ten operand streams
when the physical memory is held fixed?

One pool allocation (the same physical pages for every case); the ten operands of the bench step
(fp32 theta, fp32 momentum, K = 8 bf16 workers of the 1.3B layout) are carved out of it at
start offsets given by a layout rule, and the same launch is timed for each rule. The packed
layout is re-timed between cases to show drift.

    python scripts/pool_probe.py [--iters 10] [--json out.json]
"""
from __future__ import annotations

import argparse
import json
import os
import random
import statistics
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

MB = 1 << 20


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--json", default=None)
    a = ap.parse_args()
    from evolutionarydistributedtraining_amd import _lib as L
    from evolutionarydistributedtraining_amd.layouts import gpt_1p3b
    lib = L.lib()
    dev = torch.device("cuda:0")
    P, K = gpt_1p3b().total, 8
    sizes = [P * 4, P * 4] + [P * 2] * K
    slack = 160 * MB * len(sizes)
    pool = torch.empty(sum(sizes) + slack, dtype=torch.uint8, device=dev)
    base = pool.data_ptr()
    st = L.stream_ptr(dev)

    def packed(order=None, align=2 * MB):
        order = order or list(range(len(sizes)))
        off, starts = 0, [0] * len(sizes)
        for j in order:
            off = (off + align - 1) // align * align
            starts[j] = off
            off += sizes[j]
        return starts

    def stagger(s):
        return [o + j * s for j, o in enumerate(packed())]

    def rand(seed, span=128 * MB, align=4096):
        r = random.Random(seed)
        return [o + r.randrange(0, span // align) * align for o in packed()]

    cases = {"packed": packed()}
    for s in [256, 4096, 16384, 65536, 262144, MB, 2 * MB + 4096, 8 * MB, 64 * MB, 150 * MB]:
        cases[f"stagger_{s}"] = stagger(s)
    cases["workers_first"] = packed(order=list(range(2, len(sizes))) + [0, 1])
    cases["interleave_order"] = packed(order=[2, 3, 0, 4, 5, 1, 6, 7, 8, 9])
    for seed in range(4):
        cases[f"rand4k_{seed}"] = rand(seed)
    for seed in range(2):
        cases[f"rand2m_{seed}"] = rand(100 + seed, align=2 * MB)

    # seed every byte once (theta/momentum finite, workers near theta): bf16 1.0 / fp32 pattern
    pool.view(torch.int16).fill_(0x3C00)   # bf16 0.0078 / fp32 pairs ~ small finite numbers

    def run(starts):
        assert max(s + z for s, z in zip(starts, sizes)) <= pool.numel()
        th, mo = base + starts[0], base + starts[1]
        arr = (L.ctypes.c_void_p * K)(*[base + s for s in starts[2:]])
        f = lambda: lib.edt_outer_step(L.ctypes.c_void_p(th), 0, arr, 1, K, L.ctypes.c_void_p(mo), 1, P,
                                       0.7, 0.9, 1, st)
        assert f() == 0
        torch.cuda.synchronize()
        evs = [torch.cuda.Event(enable_timing=True) for _ in range(2 * a.iters)]
        for i in range(a.iters):
            evs[2 * i].record()
            f()
            evs[2 * i + 1].record()
        torch.cuda.synchronize()
        return statistics.median(evs[2 * i].elapsed_time(evs[2 * i + 1]) for i in range(a.iters))

    res = {}
    for name, starts in cases.items():
        t = run(starts)
        t0 = run(cases["packed"])
        res[name] = {"ms": round(t, 4), "packed_ms": round(t0, 4), "TBps": round(32 * P / t / 1e9, 3)}
        print(name, res[name], flush=True)
    out = {"P": P, "K": K, "pool_bytes": pool.numel(), "cases": res}
    print(json.dumps(out))
    if a.json:
        with open(a.json, "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
