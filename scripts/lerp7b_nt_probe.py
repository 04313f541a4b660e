"""Ordinary vs non-temporal stores for the two-parent streaming merges, interleaved on the same
buffers (the pair SLERP's lineage pass gained from nt stores at 7B, 7.06 -> 6.62 ms;
does lerp, and does the EDT-LM pair merge?). Two builds of the same sources: the shipped one
(build_variants/default.so) and EDT_NT_RMW=1 + EDT_NT_STORES=1 (build_variants/nt_rmw_st.so:
non-temporal stores of every merge output). Sizes: the 1.3B layout and the 7.07B body.

    python scripts/kernel_variants.py --build --variants default,nt_rmw_st      # here (no GPU)
    python scripts/lerp7b_nt_probe.py > profiles/r06_lerp_nt_probe.json        # GPU box

One JSON line per (op, size): median ms per variant over interleaved rounds, the TB/s of the
algorithmic bytes, and whether the outputs are bit-identical across the variants."""
import ctypes
import json
import os
import statistics
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from evolutionarydistributedtraining_amd import _lib as L  # noqa: E402

VDIR = os.path.join(ROOT, "build_variants")
VARIANTS = ("default", "nt_rmw_st")
SIZES = {"gpt_1p3b": 1315723264, "qwen2p5_7b_body": 7070619136}


def _bind(name):
    lib = ctypes.CDLL(os.path.join(VDIR, f"{name}.so"))
    lerp = lib.edt_lerp
    lerp.restype = ctypes.c_int
    lerp.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_int, ctypes.c_int,
                     ctypes.c_uint64, ctypes.c_double, ctypes.c_void_p]
    pm = lib.edt_pair_merge_to
    pm.restype = ctypes.c_int
    pm.argtypes = [ctypes.c_void_p] * 4 + [ctypes.c_int, ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p,
                                           ctypes.c_int, ctypes.c_uint64, ctypes.c_double, ctypes.c_double, ctypes.c_int,
                                           ctypes.c_void_p]
    return lerp, pm


def _time(calls, rounds=5, per=3):
    times = {n: [] for n in calls}
    for n, f in calls.items():
        assert f() == 0, n
    torch.cuda.synchronize()
    for _ in range(rounds):
        for n, f in calls.items():
            for _ in range(per):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                f()
                e1.record()
                torch.cuda.synchronize()
                times[n].append(e0.elapsed_time(e1))
    return {n: statistics.median(v) for n, v in times.items()}


def main():
    dev = torch.device("cuda:0")
    st = L.stream_ptr(dev)
    fns = {n: _bind(n) for n in VARIANTS}
    bf = torch.bfloat16
    for lname, P in SIZES.items():
        # lerp(0.5): two bf16 parents read, one bf16 child written (6 B per element)
        a = torch.empty(P, dtype=bf, device=dev).normal_(0, 0.02)
        b = torch.empty(P, dtype=bf, device=dev).normal_(0, 0.02)
        outs = {n: torch.empty(P, dtype=bf, device=dev) for n in VARIANTS}
        calls = {n: (lambda f=fns[n][0], o=outs[n]: f(a.data_ptr(), b.data_ptr(), 1, o.data_ptr(), 1, 1, P, 0.5, st))
                 for n in VARIANTS}
        ms = _time(calls)
        same = torch.equal(outs[VARIANTS[0]].view(torch.int16), outs[VARIANTS[1]].view(torch.int16))
        print(json.dumps({"op": "lerp", "layout": lname, "P": P, "bytes_per_elem": 6,
                          "median_ms": {n: round(v, 4) for n, v in ms.items()},
                          "TBps": {n: round(6 * P / v / 1e9, 3) for n, v in ms.items()}, "bits_identical": same}),
              flush=True)
        del outs, calls
        # the EDT-LM child: four bf16 parents read, child written, momentum read + written (14 B)
        m1 = torch.empty(P, dtype=bf, device=dev).normal_(0, 0.02)
        m2 = torch.empty(P, dtype=bf, device=dev).normal_(0, 0.02)
        mom_in = torch.empty(P, dtype=bf, device=dev).normal_(0, 1e-3)
        res = {n: (torch.empty(P, dtype=bf, device=dev), torch.empty(P, dtype=bf, device=dev)) for n in VARIANTS}
        calls = {n: (lambda f=fns[n][1], o=res[n]: f(a.data_ptr(), b.data_ptr(), m1.data_ptr(), m2.data_ptr(), 1,
                                                      o[0].data_ptr(), 1, mom_in.data_ptr(), o[1].data_ptr(), 1, P,
                                                      0.7, 0.9, 1, st)) for n in VARIANTS}
        ms = _time(calls)
        same = all(torch.equal(res[VARIANTS[0]][i].view(torch.int16), res[VARIANTS[1]][i].view(torch.int16))
                   for i in range(2))
        print(json.dumps({"op": "pair_merge", "layout": lname, "P": P, "bytes_per_elem": 14,
                          "median_ms": {n: round(v, 4) for n, v in ms.items()},
                          "TBps": {n: round(14 * P / v / 1e9, 3) for n, v in ms.items()}, "bits_identical": same}),
              flush=True)
        del a, b, m1, m2, mom_in, res, calls
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
