"""A/B sweep of build-time variants of the fused outer-step kernel, interleaved in one process.

    python scripts/kernel_variants.py --build            # here: hipcc the variants into build/variants/
    python scripts/kernel_variants.py --rounds 5         # on the GPU box: time them

Each variant is the same sources (evolutionarydistributedtraining_amd/csrc/*.hip) built with
different -D tunables; each is loaded as its own ctypes library and timed with HIP events on the
1.3B-parameter, K=8 bf16-worker, fp32-master configuration of bench.py.
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import statistics
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
VDIR = os.path.join(ROOT, "build_variants")      # travels to the GPU box (./build does not)

NT = ["-DEDT_NT_LOADS=1"]
VARIANTS = {
    "default": [],                                             # the shipped tunables
    "base": ["-DEDT_BLOCKS_PER_CU=8", "-DEDT_NT_LOADS=0"],     # round-1 first build
    "bpc64": ["-DEDT_BLOCKS_PER_CU=64", "-DEDT_NT_LOADS=0"],
    "bpc6_nt": ["-DEDT_BLOCKS_PER_CU=6"] + NT,
    "bpc12_nt": ["-DEDT_BLOCKS_PER_CU=12"] + NT,
    "bpc24_nt": ["-DEDT_BLOCKS_PER_CU=24"] + NT,
    "bpc64_nt": ["-DEDT_BLOCKS_PER_CU=64"] + NT,
    "bpc256_nt": ["-DEDT_BLOCKS_PER_CU=256"] + NT,
    "oneshot_nt": ["-DEDT_BLOCKS_PER_CU=0"] + NT,
    "oneshot": ["-DEDT_BLOCKS_PER_CU=0", "-DEDT_NT_LOADS=0"],
    "w8_bpc64_nt": ["-DEDT_BLOCKS_PER_CU=64", "-DEDT_MIN_WAVES=8"] + NT,
    "w8_oneshot_nt": ["-DEDT_BLOCKS_PER_CU=0", "-DEDT_MIN_WAVES=8"] + NT,
}


SLERP_VARIANTS = {"s_default": [],
                  # explicit flags, independent of the shipped defaults
                  "s_plain": ["-DEDT_NT_SLERP=0", "-DEDT_SLERP_COEF_BLOCK=0"],
                  "s_nt": ["-DEDT_NT_SLERP=1", "-DEDT_SLERP_COEF_BLOCK=0"],
                  "s_coefblk": ["-DEDT_NT_SLERP=0", "-DEDT_SLERP_COEF_BLOCK=1"],
                  "s_nt_coefblk": ["-DEDT_NT_SLERP=1", "-DEDT_SLERP_COEF_BLOCK=1"],
                  "s_bpc32_nt": ["-DEDT_SLERP_BPC=32", "-DEDT_NT_SLERP=1"],
                  "s_bpc8_nt": ["-DEDT_SLERP_BPC=8", "-DEDT_NT_SLERP=1"]}
# XCD-aware block order (edt_common.h xcd_block): runs of M consecutive tiles per XCD
VARIANTS.update({f"xcd{m}": [f"-DEDT_XCD_RUN={m}"] for m in (2, 8, 64, 512)})
VARIANTS["xcd_full"] = ["-DEDT_XCD_RUN=-1"]
# speculative SLERP pass: k consecutive chunks per workgroup in address order (EDT_SLERP_SPEC_CONTIG)
VARIANTS.update({f"spec_c{k}": [f"-DEDT_SLERP_SPEC_CONTIG={k}"] for k in (1, 2, 3, 4)})
VARIANTS.update({f"spec_b{b}": [f"-DEDT_SLERP_SPEC_BPC={b}"] for b in (32, 64, 128, 192)})
VARIANTS.update({"lerp_nt": ["-DEDT_NT_LERP=1"], "nt0": ["-DEDT_NT_LOADS=0"],
                 "bpc32_nt0": ["-DEDT_BLOCKS_PER_CU=32", "-DEDT_NT_LOADS=0"]})


def run_stream_ops(names, rounds, iters):
    """lerp (1.3B bf16, 6 B/elem) and pair merge (1.3B bf16, 14 B/elem) per variant library."""
    import torch
    from evolutionarydistributedtraining_amd import _lib as L
    from evolutionarydistributedtraining_amd.layouts import gpt_1p3b
    dev = torch.device("cuda:0")
    P = gpt_1p3b().total
    bf = torch.bfloat16
    a = (torch.randn(P, device=dev) * 0.02).to(bf)
    b = (torch.randn(P, device=dev) * 0.02).to(bf)
    m1 = (a.float() + 1e-3).to(bf)
    m2 = (b.float() + 1e-3).to(bf)
    out = torch.empty(P, dtype=bf, device=dev)
    mom = torch.zeros(P, dtype=bf, device=dev)
    st = L.stream_ptr(dev)
    Pp = L.ptr
    cases = {}
    for n in names:
        lib = ctypes.CDLL(os.path.join(VDIR, f"{n}.so"))
        for name, res, args in L.SIGNATURES:
            f = getattr(lib, name)
            f.restype, f.argtypes = res, args
        cases[f"{n}/lerp"] = (6, lambda lib=lib: lib.edt_lerp(Pp(a), Pp(b), 1, Pp(out), 1, 1, P, 0.5, st))
        cases[f"{n}/pair"] = (14, lambda lib=lib: lib.edt_pair_merge(Pp(a), Pp(b), Pp(m1), Pp(m2), 1, Pp(out), 1,
                                                                     Pp(mom), 1, P, 0.7, 0.9, 1, st))
    times = {k: [] for k in cases}
    for k, (_, f) in cases.items():
        assert f() == 0
    torch.cuda.synchronize()
    for _ in range(rounds):
        for k, (_, f) in cases.items():
            evs = [torch.cuda.Event(enable_timing=True) for _ in range(2 * iters)]
            for i in range(iters):
                evs[2 * i].record()
                f()
                evs[2 * i + 1].record()
            torch.cuda.synchronize()
            times[k] += [evs[2 * i].elapsed_time(evs[2 * i + 1]) for i in range(iters)]
    res = {k: {"median_ms": round(statistics.median(v), 4),
               "TBps": round(cases[k][0] * P / statistics.median(v) / 1e9, 3)} for k, v in times.items()}
    print(json.dumps({"op": "stream", "P": P, "variants": res}, indent=1))
VARIANTS.update(SLERP_VARIANTS)
VARIANTS.update({"f32_nt": ["-DEDT_NT_F32=1"], "f32_bpc64": ["-DEDT_BLOCKS_PER_CU=64"],
                 "f32_bpc32": ["-DEDT_BLOCKS_PER_CU=32"], "f32_oneshot": ["-DEDT_BLOCKS_PER_CU=0"],
                 "f32_nt_bpc64": ["-DEDT_NT_F32=1", "-DEDT_BLOCKS_PER_CU=64"],
                 "f32_w2": ["-DEDT_MIN_WAVES=2"],
                 "f32_nt_oneshot": ["-DEDT_NT_F32=1", "-DEDT_BLOCKS_PER_CU=0"],
                 "f32_nt_ntst": ["-DEDT_NT_F32=1", "-DEDT_NT_STORES=1"],
                 "f32_nt_bpc128": ["-DEDT_NT_F32=1", "-DEDT_BLOCKS_PER_CU=128"]})
VARIANTS.update({f"pop{i}": [f"-DEDT_POP_ITERS={i}"] for i in (1, 2, 8, 16)})
VARIANTS["r5ntst"] = []            # r5: the in-tree build after EDT_NT_SLERP_STORES (copied, not rebuilt)
VARIANTS.update({"default": [], "f32_ntst": ["-DEDT_NT_STORES=1"], "nt_rmw": ["-DEDT_NT_RMW=1"],
                 "nt_rmw_st": ["-DEDT_NT_RMW=1", "-DEDT_NT_STORES=1"],
                 "s_bpc1024": ["-DEDT_SLERP_BPC=1024"], "s_bpc4096": ["-DEDT_SLERP_BPC=4096"]})
VARIANTS.update({"split0": ["-DEDT_SPLIT_HALVES=0"], "split1": ["-DEDT_SPLIT_HALVES=1"],
                 "split1_nt0": ["-DEDT_SPLIT_HALVES=1", "-DEDT_NT_LOADS=0"]})
VARIANTS.update({f"li{i}": [f"-DEDT_LIST_ITERS={i}"] for i in (1, 2, 4, 8, 16)})
VARIANTS.update({"s_grid0": ["-DEDT_SLERP_GRID=0"], "s_grid1": ["-DEDT_SLERP_GRID=1"],
                 "s_grid1_nt0": ["-DEDT_SLERP_GRID=1", "-DEDT_NT_SLERP=0"],
                 "s_spec64": ["-DEDT_SLERP_SPEC_BPC=64"], "s_spec1024": ["-DEDT_SLERP_SPEC_BPC=1024"],
                 "s_spec16": ["-DEDT_SLERP_SPEC_BPC=16"], "s_gram1": ["-DEDT_SLERP_GRAM_GRID=1"],
                 "s_tile2k": ["-DEDT_SLERP_TPC=1", "-DEDT_SLERP_SPEC_BPC=1048576"],
                 "s_tile4k": ["-DEDT_SLERP_TPC=2", "-DEDT_SLERP_SPEC_BPC=1048576"],
                 "s_tile8k": ["-DEDT_SLERP_TPC=4", "-DEDT_SLERP_SPEC_BPC=1048576"],
                 "s_tile16k": ["-DEDT_SLERP_TPC=8", "-DEDT_SLERP_SPEC_BPC=1048576"]})
VARIANTS.update({"s_nt0": ["-DEDT_NT_SLERP=0"], "s_rev": ["-DEDT_SLERP_BLEND_REV=1"],
                 "s_rev_nt0": ["-DEDT_SLERP_BLEND_REV=1", "-DEDT_NT_SLERP=0"]})


def run_list(names, rounds, iters, wdt="bf16"):
    """Flat-arena vs tensor-list outer step (gpt_1p3b as 292 separate tensors per model, K = 8
    workers, fp32 theta + momentum) per variant library."""
    import torch
    from evolutionarydistributedtraining_amd import _lib as L
    from evolutionarydistributedtraining_amd.layouts import gpt_1p3b
    dev = torch.device("cuda:0")
    lay = gpt_1p3b()
    P, K, T = lay.total, 8, len(lay)
    theta = torch.randn(P, device=dev) * 0.02
    mom = torch.zeros(P, device=dev)
    workers = [(theta + torch.randn(P, device=dev) * 1e-3).to(torch.bfloat16 if wdt == "bf16" else torch.float32)
               for _ in range(K)]
    wc = L.dtype_code(workers[0])
    bpe = K * workers[0].element_size() + 16
    th_t = [v.clone() for v in lay.views(theta)]
    mo_t = [v.clone() for v in lay.views(mom)]
    w_t = [[v.clone() for v in lay.views(w)] for w in workers]
    st = L.stream_ptr(dev)
    Pp = L.ptr
    numel = (ctypes.c_uint64 * T)(*lay.numels)
    a_th, a_mo = L.ptr_array(th_t), L.ptr_array(mo_t)
    a_w = L.ptr_array([t for w in w_t for t in w])
    a_flat = L.ptr_array(workers)
    ws = torch.empty(1 << 20, dtype=torch.uint8, device=dev)
    one_th, one_mo = L.ptr_array([theta]), L.ptr_array([mom])     # the flat arenas as a 1-tensor list
    one_n = (ctypes.c_uint64 * 1)(P)
    # the flat arenas as the 292-tensor list of their views (same memory as flat, per-tensor chunks)
    v_th, v_mo = L.ptr_array(lay.views(theta)), L.ptr_array(lay.views(mom))
    v_w = L.ptr_array([t for w in workers for t in lay.views(w)])
    cases = {}
    for n in names:
        lib = ctypes.CDLL(os.path.join(VDIR, f"{n}.so"))
        for name, res, args in L.SIGNATURES:
            f = getattr(lib, name)
            f.restype, f.argtypes = res, args
        cases[f"{n}/flat"] = lambda lib=lib: lib.edt_outer_step(Pp(theta), 0, a_flat, wc, K, Pp(mom), 1, P, 0.7, 0.9,
                                                                1, st)
        cases[f"{n}/list"] = lambda lib=lib: lib.edt_outer_step_list(a_th, 0, a_w, wc, K, a_mo, 1, numel, T, 0.7, 0.9,
                                                                     1, Pp(ws), ws.numel(), st)
        cases[f"{n}/flat_as_list1"] = lambda lib=lib: lib.edt_outer_step_list(one_th, 0, a_flat, wc, K, one_mo, 1,
                                                                              one_n, 1, 0.7, 0.9, 1, Pp(ws),
                                                                              ws.numel(), st)
        cases[f"{n}/flat_as_views"] = lambda lib=lib: lib.edt_outer_step_list(v_th, 0, v_w, wc, K, v_mo, 1, numel, T,
                                                                              0.7, 0.9, 1, Pp(ws), ws.numel(), st)
    times = {k: [] for k in cases}
    for f in cases.values():
        assert f() == 0
    torch.cuda.synchronize()
    for _ in range(rounds):
        for k, f in cases.items():
            evs = [torch.cuda.Event(enable_timing=True) for _ in range(2 * iters)]
            for i in range(iters):
                evs[2 * i].record()
                f()
                evs[2 * i + 1].record()
            torch.cuda.synchronize()
            times[k] += [evs[2 * i].elapsed_time(evs[2 * i + 1]) for i in range(iters)]
    res = {k: {"median_ms": round(statistics.median(v), 4), "TBps": round(bpe * P / statistics.median(v) / 1e9, 3)}
           for k, v in times.items()}
    print(json.dumps({"op": "list", "P": P, "tensors": T, "workers": wdt, "variants": res}, indent=1))


def run_slerp(names, rounds, layout_name):
    """Qwen2.5-7B-body-sized SLERP (bf16 in/out) per variant library, each pass timed on its own
    (stats = chunk sums, 4 B/elem read; blend = 4 B read + 2 B written; spec = the speculative
    stats+lerp pass, 6 B/elem) and the whole merges: two-pass (far parents) and speculative
    (lineage parents, every tensor in the lerp branch)."""
    import torch
    from evolutionarydistributedtraining_amd import _lib as L
    from evolutionarydistributedtraining_amd import ops
    from evolutionarydistributedtraining_amd.layouts import LAYOUTS
    dev = torch.device("cuda:0")
    lay = LAYOUTS[layout_name]()
    P = lay.total
    bf = torch.bfloat16
    v0 = torch.empty(P, dtype=bf, device=dev)
    v1 = torch.empty(P, dtype=bf, device=dev)
    v2 = torch.empty(P, dtype=bf, device=dev)        # lineage partner of v0
    for s0 in range(0, P, 1 << 28):
        e = min(P, s0 + (1 << 28))
        x = torch.randn(e - s0, device=dev) * 0.02
        v0[s0:e] = x.to(bf)
        v1[s0:e] = (x + torch.randn(e - s0, device=dev) * 1e-3).to(bf)
        v2[s0:e] = (x + torch.randn(e - s0, device=dev) * 1e-4).to(bf)
        del x
    out = torch.empty(P, dtype=bf, device=dev)
    plan = ops.make_slerp_plan(lay.offsets, dev, chunk_elems=int(os.environ.get("EDT_VARIANT_CHUNK", 1 << 16)))
    redo = torch.zeros(plan.nseg, dtype=torch.int32, device=dev)
    t = torch.full((len(lay),), 0.5, dtype=torch.float64, device=dev)
    stream = L.stream_ptr(dev)
    libs = {}
    for n in names:
        lib = ctypes.CDLL(os.path.join(VDIR, f"{n}.so"))
        for name, res, args in L.SIGNATURES:
            f = getattr(lib, name)
            f.restype, f.argtypes = res, args
        libs[n] = lib
    P_ = L.ptr
    cases = {}
    for n in names:
        lib = libs[n]
        cases[f"{n}/stats"] = (4, lambda lib=lib: lib.edt_slerp_stats(P_(v0), P_(v1), 1, P_(plan.chunks), plan.nchunks,
                                                                       P_(plan.partial), stream))
        cases[f"{n}/blend"] = (6, lambda lib=lib: lib.edt_slerp_blend(P_(v0), P_(v1), 1, P_(out), 1, P_(plan.chunks),
                                                                       plan.nchunks, P_(plan.coef), stream))
        cases[f"{n}/two_pass_far"] = (6, lambda lib=lib: lib.edt_slerp_merge(
            P_(v0), P_(v1), 1, P_(out), 1, P_(plan.chunks), plan.nchunks, P_(plan.seg_first), plan.nseg, P_(t),
            0.9995, 1e-8, P_(plan.partial), P_(plan.coef), P_(plan.dots), stream))
        cases[f"{n}/speculative_lineage"] = (6, lambda lib=lib: lib.edt_slerp_merge_speculative(
            P_(v0), P_(v2), 1, P_(out), 1, P_(plan.chunks), plan.nchunks, P_(plan.seg_first), plan.nseg, P_(t),
            0.9995, 1e-8, P_(plan.partial), P_(plan.coef), P_(plan.dots), P_(redo), P, stream))
    times = {k: [] for k in cases}
    for k, (_, f) in cases.items():
        assert f() == 0, k
    torch.cuda.synchronize()
    for _ in range(rounds):
        for k, (_, f) in cases.items():
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            f()
            b.record()
            torch.cuda.synchronize()
            times[k].append(a.elapsed_time(b))
    res = {k: {"median_ms": round(statistics.median(v), 3),
               "TBps": round(cases[k][0] * P / statistics.median(v) / 1e9, 3)} for k, v in times.items()}
    # results must not depend on the grid: every variant's two-pass output is compared
    outs = {}
    for n in names:
        cases[f"{n}/two_pass_far"][1]()
        outs[n] = out.clone()
    torch.cuda.synchronize()
    ref = outs[names[0]]
    res["identical_outputs"] = all(torch.equal(o.view(torch.int16), ref.view(torch.int16)) for o in outs.values())
    print(json.dumps({"layout": layout_name, "P": P, "op": "slerp", "chunks": plan.nchunks, "variants": res},
                     indent=1))


def run_slerp_pop(names, rounds, layout_name="gpt_1p3b", P_members=8):
    """One resident SLERP generation (edt_slerp_population: Gram pass + per-child blends) over
    8 bf16 members of the layout, per variant library."""
    import torch
    from evolutionarydistributedtraining_amd import _lib as L
    from evolutionarydistributedtraining_amd import ops
    from evolutionarydistributedtraining_amd.layouts import LAYOUTS
    dev = torch.device("cuda:0")
    lay = LAYOUTS[layout_name]()
    P = lay.total
    g = torch.Generator(device=dev).manual_seed(2)
    mem = [(torch.randn(P, device=dev, generator=g) * 0.02).bfloat16() for _ in range(P_members)]
    outs = [torch.empty(P, dtype=torch.bfloat16, device=dev) for _ in range(P_members)]
    pairs = [(i, (i + 3) % P_members) for i in range(P_members)]
    t = torch.full((len(lay),), 0.5, dtype=torch.float64, device=dev)
    stream = L.stream_ptr(dev)
    plans = {ce: ops.make_slerp_plan(lay.offsets, dev, chunk_elems=ce) for ce in (1 << 14, 1 << 16)}
    # the Gram rows AND the row scratch the pass folds into them (edt_slerp_population_gram_doubles)
    grams = {ce: torch.empty(int(L.lib().edt_slerp_population_gram_doubles(P_members, pl.nchunks)), dtype=torch.float64,
                             device=dev) for ce, pl in plans.items()}
    coef = torch.empty(P_members * len(lay) * 2, dtype=torch.float32, device=dev)
    flat = (ctypes.c_int32 * (2 * P_members))(*[x for p in pairs for x in p])
    am, ao = L.ptr_array(mem), L.ptr_array(outs)
    cases = {}
    for n in names:
        lib = ctypes.CDLL(os.path.join(VDIR, f"{n}.so"))
        for name, res, args in L.SIGNATURES:
            f = getattr(lib, name)
            f.restype, f.argtypes = res, args
        for ce, pl in plans.items():
            cases[f"{n}/chunk{ce >> 10}k"] = (lambda lib=lib, pl=pl, gr=grams[ce]: lib.edt_slerp_population(
                am, P_members, 1, flat, P_members, ao, 1, L.ptr(pl.chunks), pl.nchunks, L.ptr(pl.seg_first),
                pl.nseg, L.ptr(t), 0.9995, 1e-8, L.ptr(gr), L.ptr(coef), None, stream))
    times = {k: [] for k in cases}
    for f in cases.values():
        assert f() == 0
    torch.cuda.synchronize()
    for _ in range(rounds):
        for k, f in cases.items():
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            f()
            b.record()
            torch.cuda.synchronize()
            times[k].append(a.elapsed_time(b))
    res = {k: {"median_ms": round(statistics.median(v), 3),
               "moved_TBps": round(8 * P * P_members / statistics.median(v) / 1e9, 3)} for k, v in times.items()}
    print(json.dumps({"layout": layout_name, "P": P, "members": P_members, "op": "slerp_pop", "variants": res},
                     indent=1))


def run_pair_pop(names, rounds, layout_name="gpt_1p3b"):
    """One resident EDT-LM generation (edt_pair_merge_population, 8 children of 6 distinct parents,
    bf16 members and momenta) per variant library."""
    import torch
    from evolutionarydistributedtraining_amd import _lib as L
    from evolutionarydistributedtraining_amd.layouts import LAYOUTS
    dev = torch.device("cuda:0")
    n = LAYOUTS[layout_name]().total
    bf = torch.bfloat16
    g = torch.Generator(device=dev).manual_seed(3)
    M = 8
    base = [(torch.randn(n, device=dev, generator=g) * 0.02).to(bf) for _ in range(M)]
    trained = [(b.float() + 1e-3).to(bf) for b in base]
    moms = [(torch.randn(n, device=dev, generator=g) * 1e-3).to(bf) for _ in range(M)]
    pairs = [(0, 1), (1, 2), (2, 0), (3, 4), (4, 5), (5, 3), (0, 3), (1, 4)]   # 6 distinct parents
    outs = [torch.empty(n, dtype=bf, device=dev) for _ in pairs]
    omom = [torch.empty(n, dtype=bf, device=dev) for _ in pairs]
    C = len(pairs)
    arr = lambda ts: (ctypes.c_void_p * C)(*[t.data_ptr() for t in ts])
    a_b1, a_b2 = arr([base[i] for i, _ in pairs]), arr([base[j] for _, j in pairs])
    a_m1, a_m2 = arr([trained[i] for i, _ in pairs]), arr([trained[j] for _, j in pairs])
    a_out, a_min, a_mout = arr(outs), arr([moms[i] for i, _ in pairs]), arr(omom)
    has = (ctypes.c_int32 * C)(*([1] * C))
    stream = L.stream_ptr(dev)
    cases = {}
    for nm in names:
        lib = ctypes.CDLL(os.path.join(VDIR, f"{nm}.so"))
        for name, res, args in L.SIGNATURES:
            f = getattr(lib, name)
            f.restype, f.argtypes = res, args
        cases[nm] = (lambda lib=lib: lib.edt_pair_merge_population(a_b1, a_b2, a_m1, a_m2, 1, a_out, 1, a_min, a_mout,
                                                                   has, C, n, 0.7, 0.9, 1, stream))
    times = {k: [] for k in cases}
    for k, f in cases.items():
        assert f() == 0
    torch.cuda.synchronize()
    for _ in range(rounds):
        for k, f in cases.items():
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            assert f() == 0
            b.record()
            torch.cuda.synchronize()
            times[k].append(a.elapsed_time(b))
    floor = n * (6 * 2 * 2 + 6 * 2 + C * 2 * 2)     # distinct parents' base + trained, donor moms, children
    res = {k: {"median_ms": round(statistics.median(v), 4),
               "floor_TBps": round(floor / statistics.median(v) / 1e9, 3)} for k, v in times.items()}
    print(json.dumps({"op": "pair_pop", "n": n, "variants": res}, indent=1))


def build(names):
    from evolutionarydistributedtraining_amd.build import build_library
    os.makedirs(VDIR, exist_ok=True)
    for n in names:
        out = os.path.join(VDIR, f"{n}.so")
        build_library(force=True, extra_flags=VARIANTS[n], out=out)
        print("built", out)


def run(names, rounds, iters, layout_name, k, tdt="f32", wdt="bf16", place=True):
    import torch
    from evolutionarydistributedtraining_amd import _lib as L
    from evolutionarydistributedtraining_amd.layouts import LAYOUTS
    dev = torch.device("cuda:0")
    P = LAYOUTS[layout_name]().total
    DT = {"f32": torch.float32, "bf16": torch.bfloat16}
    theta = (torch.randn(P, device=dev) * 0.02).to(DT[tdt])
    workers = [(theta.float() + torch.randn(P, device=dev) * 1e-3).to(DT[wdt]) for _ in range(k)]
    mom = torch.zeros(P, device=dev, dtype=DT[tdt])
    if place:       # the bench's momentum placement (placement.py), so variants compare on a good one
        from evolutionarydistributedtraining_amd.placement import place_momentum
        mom, rep = place_momentum(theta, workers, mom)
        print("momentum placement", rep, flush=True)
    libs = {}
    for n in names:
        lib = ctypes.CDLL(os.path.join(VDIR, f"{n}.so"))
        f = lib.edt_outer_step
        f.restype = ctypes.c_int
        f.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.POINTER(ctypes.c_void_p), ctypes.c_int,
                      ctypes.c_int, ctypes.c_void_p, ctypes.c_int, ctypes.c_uint64, ctypes.c_double,
                      ctypes.c_double, ctypes.c_int, ctypes.c_void_p]
        libs[n] = f
    arr = L.ptr_array(workers)
    stream = L.stream_ptr(dev)
    bw, bg = (2 if wdt == "bf16" else 4), (2 if tdt == "bf16" else 4)
    bytes_per = k * bw + 4 * bg
    times = {n: [] for n in names}

    def launch(f):
        rc = f(ctypes.c_void_p(theta.data_ptr()), L.dtype_code(theta), arr, L.dtype_code(workers[0]), k,
               ctypes.c_void_p(mom.data_ptr()), 1, P, 0.7, 0.9, 1, stream)
        assert rc == 0
    for n in names:                       # warm-up, first-step buffer init
        launch(libs[n])
    torch.cuda.synchronize()
    for r in range(rounds):
        for n in names:
            evs = [torch.cuda.Event(enable_timing=True) for _ in range(2 * iters)]
            for i in range(iters):
                evs[2 * i].record()
                launch(libs[n])
                evs[2 * i + 1].record()
            torch.cuda.synchronize()
            times[n] += [evs[2 * i].elapsed_time(evs[2 * i + 1]) for i in range(iters)]
    res = {}
    for n in names:
        med = statistics.median(times[n])
        res[n] = {"median_ms": round(med, 4), "min_ms": round(min(times[n]), 4),
                  "TBps": round(bytes_per * P / med / 1e9, 3)}
    print(json.dumps({"layout": layout_name, "K": k, "theta": tdt, "workers": wdt, "variants": res}, indent=1))


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--build", action="store_true")
    ap.add_argument("--variants", default=",".join(VARIANTS))
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--layout", default="gpt_1p3b")
    ap.add_argument("--k", type=int, default=8)
    ap.add_argument("--tdt", default="f32")
    ap.add_argument("--wdt", default="bf16")
    ap.add_argument("--op", default="outer", choices=["outer", "slerp", "slerp_pop", "stream", "list", "pair_pop"])
    a = ap.parse_args()
    names = a.variants.split(",")
    if a.build:
        build(names)
    elif a.op == "stream":
        run_stream_ops(names, a.rounds, a.iters)
    elif a.op == "list":
        run_list(names, a.rounds, a.iters, a.wdt)
    elif a.op == "pair_pop":
        run_pair_pop(names, a.rounds)
    elif a.op == "slerp_pop":
        run_slerp_pop(names, a.rounds)
    elif a.op == "slerp":
        run_slerp(names, a.rounds, a.layout if a.layout != "gpt_1p3b" else "qwen2p5_7b_body")
    else:
        run(names, a.rounds, a.iters, a.layout, a.k, a.tdt, a.wdt)
