"""Sweep: the fused outer step (flat launch, 1.3B, K = 8 bf16 workers, fp32 theta + momentum)
with operand j's arena starting j * S bytes past an allocation boundary, for several S.
Each case gets fresh arenas (freed after), and the unshifted arenas are re-timed beside it.

    python scripts/shift_sweep.py [--shifts 0,256,4096,4352,...] [--iters 10]
"""
from __future__ import annotations

import argparse
import json
import os
import statistics
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shifts", default="256,1024,2048,4096,4352,8192,8448,16640,65792,262400,1052672")
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--wdt", default="bf16")
    a = ap.parse_args()
    from evolutionarydistributedtraining_amd import _lib as L
    from evolutionarydistributedtraining_amd.layouts import gpt_1p3b
    lib = L.lib()
    dev = torch.device("cuda:0")
    P, K = gpt_1p3b().total, 8
    wdt = {"bf16": torch.bfloat16, "f32": torch.float32}[a.wdt]
    st = L.stream_ptr(dev)
    g = torch.Generator(device=dev).manual_seed(3)
    base = torch.randn(P, device=dev, generator=g) * 0.02

    def arenas(shift):
        out, keep = [], []
        for j, (dt, n) in enumerate([(torch.float32, P), (torch.float32, P)] + [(wdt, P)] * K):
            es = torch.empty(0, dtype=dt).element_size()
            buf = torch.empty(n * es + j * shift + 256, dtype=torch.uint8, device=dev)
            v = buf[j * shift:j * shift + n * es].view(dt)
            keep.append(buf)
            out.append(v)
        out[0].copy_(base)
        out[1].zero_()
        for k in range(K):
            out[2 + k].copy_(base + 1e-3 * (k + 1))
        return out, keep

    def timeit(ops_):
        th, mo, ws = ops_[0], ops_[1], ops_[2:]
        arr = L.ptr_array(ws)
        f = lambda: lib.edt_outer_step(L.ptr(th), 0, arr, L.dtype_code(wdt), K, L.ptr(mo), 1, P, 0.7, 0.9, 1, st)
        assert f() == 0
        torch.cuda.synchronize()
        evs = [torch.cuda.Event(enable_timing=True) for _ in range(2 * a.iters)]
        for i in range(a.iters):
            evs[2 * i].record()
            f()
            evs[2 * i + 1].record()
        torch.cuda.synchronize()
        return statistics.median(evs[2 * i].elapsed_time(evs[2 * i + 1]) for i in range(a.iters))

    ref, keep_ref = arenas(0)
    bpe = K * ref[2].element_size() + 16
    res = {}
    for s in [int(x) for x in a.shifts.split(",")]:
        ops_, keep = arenas(s)
        t_s = timeit(ops_)
        del ops_, keep
        torch.cuda.empty_cache()
        t_0 = timeit(ref)
        res[s] = {"ms": round(t_s, 4), "ref_ms": round(t_0, 4), "TBps": round(bpe * P / t_s / 1e9, 3)}
        print(s, res[s], flush=True)
    src = torch.empty(1 << 29, dtype=torch.float32, device=dev)
    dst = torch.empty_like(src)
    dst.copy_(src)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(5):
        dst.copy_(src)
    e1.record()
    torch.cuda.synchronize()
    print(json.dumps({"wdt": a.wdt, "copy_TBps": round(5 * 2 * src.numel() * 4 / e0.elapsed_time(e1) / 1e9, 3),
                      "shifts": res}))


if __name__ == "__main__":
    main()
