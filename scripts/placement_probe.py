"""Probe: does WHERE the operands live change the fused step's speed on a given box?

One process, interleaved timing (HIP events) of the DiLoCo step on the 1.3B layout, K = 8 bf16
workers, fp32 theta + momentum, with the same values placed as
  arena      one allocation per operand (what bench.py does)
  stagger    the ten operands carved from one buffer, operand j shifted by j x (4 KiB + 256 B)
  list       292 separate allocations per operand, tensor-list launch (edt_outer_step_list)
  arena_l1   the arenas again, through the tensor-list launch as a one-tensor list
plus a plain device copy as the box's speed reference.

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
    cases = {}
    a_w = L.ptr_array(workers)
    cases["arena"] = lambda: lib.edt_outer_step(Pp(theta), 0, a_w, 1, K, Pp(mom), 1, P, 0.7, 0.9, 1, st)
    ws = torch.empty(1 << 20, dtype=torch.uint8, device=dev)
    one_th, one_mo, one_n = L.ptr_array([theta]), L.ptr_array([mom]), (ctypes.c_uint64 * 1)(P)
    cases["arena_l1"] = lambda: lib.edt_outer_step_list(one_th, 0, a_w, 1, K, one_mo, 1, one_n, 1, 0.7, 0.9, 1,
                                                        Pp(ws), ws.numel(), st)
    # staggered: one byte buffer, operand j at offset sum of sizes + j * (4096 + 256)
    sizes = [P * 4, P * 4] + [P * 2] * K
    shift = 4096 + 256
    big = torch.empty(sum(sizes) + len(sizes) * shift + 256, dtype=torch.uint8, device=dev)
    views, off = [], 0
    for j, nb in enumerate(sizes):
        off += shift
        views.append(big[off:off + nb])
        off += nb
    s_th = views[0].view(torch.float32)
    s_mo = views[1].view(torch.float32)
    s_w = [v.view(torch.bfloat16) for v in views[2:]]
    s_th.copy_(theta)
    s_mo.copy_(mom)
    for d, w in zip(s_w, workers):
        d.copy_(w)
    a_sw = L.ptr_array(s_w)
    cases["stagger"] = lambda: lib.edt_outer_step(Pp(s_th), 0, a_sw, 1, K, Pp(s_mo), 1, P, 0.7, 0.9, 1, st)
    th_t = [v.clone() for v in lay.views(theta)]
    mo_t = [v.clone() for v in lay.views(mom)]
    w_t = [[v.clone() for v in lay.views(w)] for w in workers]
    numel = (ctypes.c_uint64 * T)(*lay.numels)
    l_th, l_mo, l_w = L.ptr_array(th_t), L.ptr_array(mo_t), L.ptr_array([t for w in w_t for t in w])
    cases["list"] = lambda: lib.edt_outer_step_list(l_th, 0, l_w, 1, K, l_mo, 1, numel, T, 0.7, 0.9, 1,
                                                    Pp(ws), ws.numel(), st)
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
