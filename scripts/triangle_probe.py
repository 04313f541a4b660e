"""r6: the population's triangle layout as a mode of the needed-sums pass against the separate Gram
kernel it replaced, on the dense pair graphs that take it, interleaved on the
same members: the previous library (build_variants/default.so, with slerp_gram_kernel) and the
in-tree one (slerp_need_kernel<IDT, D, false, ODT, true>), both through edt_slerp_population (the
two-pass form, whose signature did not change), and a roulette-drawn graph (needed layout in both)
as the control. Outputs compared bit for bit across the two libraries.

    python scripts/triangle_probe.py > profiles/r06_triangle_probe.jsonl        # GPU box
"""
import ctypes
import json
import os
import statistics
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from evolutionarydistributedtraining_amd import _lib as L  # noqa: E402
from evolutionarydistributedtraining_amd import ops  # noqa: E402
from evolutionarydistributedtraining_amd.layouts import LAYOUTS  # noqa: E402
from evolutionarydistributedtraining_amd.schedule import roulette_generation_pairs  # noqa: E402

GRAPHS = {
    "k5": [(a, b) for a in range(5) for b in range(a + 1, 5)],
    "k8_28_children": [(a, b) for a in range(8) for b in range(a + 1, 8)],
    "star8": [(0, m) for m in range(1, 8)] + [(2, 3)],
    "roulette_control": [tuple(p) for p in roulette_generation_pairs(8, 1, seed=2025)[0]["pairs"]],
}


def bind(path):
    lib = ctypes.CDLL(path)
    f = lib.edt_slerp_population
    for name, res, args in L.SIGNATURES:
        if name == "edt_slerp_population":
            f.restype, f.argtypes = res, args
    g = lib.edt_slerp_population_gram_doubles
    g.restype, g.argtypes = ctypes.c_uint64, [ctypes.c_int, ctypes.c_int64]
    return f, g


def main():
    dev = torch.device("cuda:0")
    lay = LAYOUTS[os.environ.get("LAYOUT", "gpt_1p3b")]()
    P, bf, M = lay.total, torch.bfloat16, 8
    g = torch.Generator(device=dev).manual_seed(3)
    members = []
    x = torch.randn(P, generator=g, device=dev) * 0.02
    for m in range(M):
        members.append((x + torch.randn(P, generator=g, device=dev) * 0.02 * (0.005 if m % 2 else 0.5)).to(bf))
    del x
    plan = ops.make_slerp_plan(lay.offsets, dev)
    t = torch.full((len(lay),), 0.5, dtype=torch.float64, device=dev)
    libs = {"previous_gram_kernel": bind(os.path.join(ROOT, "build_variants", "default.so")),
            "needed_pass_triangle": bind(L.LIB_PATH)}
    st = L.stream_ptr(dev)
    for name, pairs in GRAPHS.items():
        Q = len(pairs)
        fp = (ctypes.c_int32 * (2 * Q))(*[v for p in pairs for v in p])
        coef = torch.empty((Q, plan.nseg, 2), dtype=torch.float32, device=dev)
        outs = {k: [torch.empty(P, dtype=bf, device=dev) for _ in range(Q)] for k in libs}
        calls = {}
        for k, (f, gd) in libs.items():
            work = torch.empty(int(gd(M, plan.nchunks)), dtype=torch.float64, device=dev)
            os_ = outs[k]
            optr = (ctypes.c_void_p * Q)(*[o.data_ptr() for o in os_])
            calls[k] = (lambda f=f, work=work, optr=optr: f(L.ptr_array(members), M, 1, fp, Q, optr, 1, L.ptr(plan.chunks),
                                                            plan.nchunks, L.ptr(plan.seg_first), plan.nseg, L.ptr(t),
                                                            0.9995, 1e-8, L.ptr(work), L.ptr(coef), None, st))
        times = {k: [] for k in libs}
        for k, c in calls.items():
            assert c() == 0, k
        torch.cuda.synchronize()
        for _ in range(5):
            for k, c in calls.items():
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                c()
                e1.record()
                torch.cuda.synchronize()
                times[k].append(e0.elapsed_time(e1))
        same = all(torch.equal(a.view(torch.int16), b.view(torch.int16))
                   for a, b in zip(outs["previous_gram_kernel"], outs["needed_pass_triangle"]))
        lay_json = ops.population_layout(pairs, M, False)
        print(json.dumps({"graph": name, "children": Q, "P": P,
                          "stats_layout": [c["stats_layout"] for c in lay_json["components"]],
                          "median_ms": {k: round(statistics.median(v), 3) for k, v in times.items()},
                          "bits_identical": same}), flush=True)
        del outs, calls, coef
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
