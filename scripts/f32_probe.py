"""Probe: why the all-fp32 DiLoCo step (48 B/elem) streams slower than the bf16-worker one.

Times the fused step on the 1.3B layout (K = 8) with the worker arenas (a) as separate
allocations, (b) carved from one buffer with staggered offsets (k x 64 KiB + k x 4 KiB), for the
library variants given, interleaved in one process.

    python scripts/f32_probe.py --variants default,base --wdt f32
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import statistics
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--variants", default="default")
    ap.add_argument("--wdt", default="f32")
    ap.add_argument("--tdt", default="f32")
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--iters", type=int, default=5)
    a = ap.parse_args()
    from evolutionarydistributedtraining_amd import _lib as L
    from evolutionarydistributedtraining_amd.layouts import gpt_1p3b
    dt = {"f32": torch.float32, "bf16": torch.bfloat16}
    wdt, tdt = dt[a.wdt], dt[a.tdt]
    dev = torch.device("cuda:0")
    P, K = gpt_1p3b().total, 8
    theta = (torch.randn(P, device=dev) * 0.02).to(tdt)
    mom = torch.zeros(P, dtype=tdt, device=dev)
    sep = [(theta.float() + 1e-3 * (k + 1)).to(wdt) for k in range(K)]
    pads = [k * (64 << 10) + k * 4096 for k in range(K)]
    es = torch.empty(0, dtype=wdt).element_size()
    big = torch.empty(K * P + sum(pads) // es + 64, dtype=wdt, device=dev)
    stag = []
    off = 0
    for k in range(K):
        off += pads[k] // es
        stag.append(big[off:off + P])
        stag[-1].copy_(sep[k])
        off += P
    st = L.stream_ptr(dev)
    libs = {}
    for n in a.variants.split(","):
        path = L.LIB_PATH if n == "shipped" else os.path.join(ROOT, "build", "variants", f"{n}.so")
        lib = ctypes.CDLL(path)
        for name, res, args in L.SIGNATURES:
            f = getattr(lib, name)
            f.restype, f.argtypes = res, args
        libs[n] = lib
    cases = {}
    for n, lib in libs.items():
        for tag, ws in (("separate", sep), ("staggered", stag)):
            arr = L.ptr_array(ws)
            cases[f"{n}/{tag}"] = (lambda lib=lib, arr=arr: lib.edt_outer_step(
                L.ptr(theta), L.dtype_code(theta), arr, L.dtype_code(wdt), K, L.ptr(mom), 1, P, 0.7, 0.9, 1, st))
    times = {k: [] for k in cases}
    for f in cases.values():
        assert f() == 0
    torch.cuda.synchronize()
    for _ in range(a.rounds):
        for k, f in cases.items():
            evs = [torch.cuda.Event(enable_timing=True) for _ in range(2 * a.iters)]
            for i in range(a.iters):
                evs[2 * i].record()
                f()
                evs[2 * i + 1].record()
            torch.cuda.synchronize()
            times[k] += [evs[2 * i].elapsed_time(evs[2 * i + 1]) for i in range(a.iters)]
    bpe = K * es + 4 * theta.element_size()
    print(json.dumps({k: {"median_ms": round(statistics.median(v), 3),
                          "TBps": round(bpe * P / statistics.median(v) / 1e9, 3)} for k, v in times.items()}))


if __name__ == "__main__":
    main()
