"""lerp at the 7B body's size (7.07e9 bf16, 6 B per element) with ordinary stores (the shipped
build, build_variants/default.so) and with non-temporal stores (build_variants/nt_rmw_st.so,
EDT_NT_STORES=1), interleaved: does the pair SLERP's store gain carry over to lerp at this size?"""
import ctypes
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from evolutionarydistributedtraining_amd import _lib as L  # noqa: E402

VDIR = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "build_variants")


def main():
    dev = torch.device("cuda:0")
    P = 7070619136
    a = torch.empty(P, dtype=torch.bfloat16, device=dev).normal_(0, 0.02)
    b = torch.empty(P, dtype=torch.bfloat16, device=dev).normal_(0, 0.02)
    out = torch.empty(P, dtype=torch.bfloat16, device=dev)
    st = L.stream_ptr(dev)
    libs = {}
    for n in ("default", "nt_rmw_st"):
        f = ctypes.CDLL(os.path.join(VDIR, f"{n}.so")).edt_lerp
        f.restype = ctypes.c_int
        f.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_int, ctypes.c_int,
                      ctypes.c_uint64, ctypes.c_double, ctypes.c_void_p]
        libs[n] = f
    times = {n: [] for n in libs}
    for n, f in libs.items():
        assert f(a.data_ptr(), b.data_ptr(), 1, out.data_ptr(), 1, 1, P, 0.5, st) == 0
    torch.cuda.synchronize()
    for _ in range(5):
        for n, f in libs.items():
            for _ in range(3):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                f(a.data_ptr(), b.data_ptr(), 1, out.data_ptr(), 1, 1, P, 0.5, st)
                e1.record()
                torch.cuda.synchronize()
                times[n].append(e0.elapsed_time(e1))
    print(json.dumps({"probe": "lerp7b_nt", "P": P, "median_ms": {n: round(statistics.median(v), 4) for n, v in times.items()},
                      "TBps": {n: round(6 * P / statistics.median(v) / 1e9, 3) for n, v in times.items()}}))


if __name__ == "__main__":
    main()
