"""Probe: does WHERE the operands live change the fused step's speed on a given box?

One process, interleaved timing (HIP events) of the DiLoCo step on the 1.3B layout, K = 8 bf16
workers, fp32 theta + momentum. Every case runs the tensor-list launch (edt_outer_step_list,
292 tensors; on par with the flat launch) over the same values, each operand placed as
  A   views of one arena per operand (what bench.py allocates)
  S   separate allocations, one per tensor
  Gx  views of one arena per operand, operand j's arena shifted by j * x bytes
and the flat launch over the arenas as the reference point, plus a plain device copy.

    python scripts/placement_probe.py [--rounds 3 --iters 5]
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
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--iters", type=int, default=5)
    a = ap.parse_args()
    from evolutionarydistributedtraining_amd import _lib as L
    from evolutionarydistributedtraining_amd.layouts import gpt_1p3b
    lib = L.lib()
    dev = torch.device("cuda:0")
    lay = gpt_1p3b()
    P, K, T = lay.total, 8, len(lay)
    st = L.stream_ptr(dev)
    Pp = L.ptr
    g = torch.Generator(device=dev).manual_seed(3)
    theta = torch.randn(P, device=dev, generator=g) * 0.02
    mom = torch.zeros(P, device=dev)
    workers = [(theta + torch.randn(P, device=dev, generator=g) * 1e-3).bfloat16() for _ in range(K)]
    ops_ = [theta, mom] + workers                       # operand j
    numel = (ctypes.c_uint64 * T)(*lay.numels)
    ws = torch.empty(1 << 20, dtype=torch.uint8, device=dev)
    keep = []

    def place(j, how):
        src = ops_[j]
        if how == "A":
            return lay.views(src)
        if how == "S":
            ts = [v.clone() for v in lay.views(src)]
            keep.append(ts)
            return ts
        shift = int(how[1:]) * j                          # "G<bytes>"
        nb = src.numel() * src.element_size()
        buf = torch.empty(nb + shift + 256, dtype=torch.uint8, device=dev)
        v = buf[shift:shift + nb].view(src.dtype)
        v.copy_(src)
        keep.append(buf)
        return lay.views(v)

    cases = {}

    def add(name, hows):
        tl = [place(j, h) for j, h in enumerate(hows)]
        a_th, a_mo = L.ptr_array(tl[0]), L.ptr_array(tl[1])
        a_w = L.ptr_array([t for w in tl[2:] for t in w])
        cases[name] = lambda: lib.edt_outer_step_list(a_th, 0, a_w, 1, K, a_mo, 1, numel, T, 0.7, 0.9, 1,
                                                      Pp(ws), ws.numel(), st)

    a_w = L.ptr_array(workers)
    cases["flat_arena"] = lambda: lib.edt_outer_step(Pp(theta), 0, a_w, 1, K, Pp(mom), 1, P, 0.7, 0.9, 1, st)
    add("list_A", ["A"] * 10)
    add("list_S", ["S"] * 10)
    add("theta_mom_S", ["S", "S"] + ["A"] * K)
    add("workers_S", ["A", "A"] + ["S"] * K)
    add("G4352", ["G4352"] * 10)
    add("G1052672", ["G1052672"] * 10)                   # 1 MiB + 4 KiB
    add("G37748736", ["G37748736"] * 10)                 # 36 MiB
    torch.cuda.empty_cache()
    src = torch.empty(1 << 29, dtype=torch.float32, device=dev)
    dst = torch.empty_like(src)
    cases["copy_4GiB"] = lambda: (dst.copy_(src), 0)[1]
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
    res = {}
    for k, v in times.items():
        med = statistics.median(v)
        nbytes = 2 * src.numel() * 4 if k.startswith("copy") else 32 * P
        res[k] = {"median_ms": round(med, 4), "TBps": round(nbytes / med / 1e9, 3)}
    print(json.dumps(res))


if __name__ == "__main__":
    main()
