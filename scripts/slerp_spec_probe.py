"""The speculative SLERP pass against lerp's identical stream on the 7B body (bf16, lineage parents:
every segment in the lerp branch, so the speculative merge is one pass of 2 reads + 1 write per
element, exactly lerp's bytes). Times, in one process on the same arenas and interleaved:
edt_lerp, edt_slerp_merge_speculative, the two-pass edt_slerp_merge (stats + blend), the
tensor-list forms over views of the same arenas (ops.slerp_list: two-pass and speculative) and the
stats pass alone (edt_slerp_stats, 4 B read per element). (r3's one-launch hold form was removed in
r4: measured slower)
HIP events on the launch stream, median over rounds. Run it under rocprofv3 (--kernel-trace
--stats, or one --pmc pass) to get the per-kernel figures.

    python scripts/slerp_spec_probe.py [--rounds 6] [--far] [--variants build_variants/slerp]

--variants DIR: also time every lib*.so in DIR (scripts/kernel_variants.py --build-slerp-slots),
each with its own workspace, interleaved with the in-tree library.
"""
import argparse
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=6)
    ap.add_argument("--far", action="store_true", help="independent parents (the SLERP branch)")
    ap.add_argument("--variants", default="")
    a = ap.parse_args()
    from evolutionarydistributedtraining_amd import _lib as L
    from evolutionarydistributedtraining_amd import ops
    from evolutionarydistributedtraining_amd.layouts import qwen2p5_7b_body
    dev = torch.device("cuda:0")
    lib = L.lib()
    lay = qwen2p5_7b_body()
    P = lay.total
    bf = torch.bfloat16
    v0 = torch.empty(P, dtype=bf, device=dev)
    v1 = torch.empty(P, dtype=bf, device=dev)
    out = torch.empty(P, dtype=bf, device=dev)
    g = torch.Generator(device=dev).manual_seed(7)
    for s0 in range(0, P, 1 << 28):
        e = min(P, s0 + (1 << 28))
        x = torch.randn(e - s0, device=dev, generator=g) * 0.02
        v0[s0:e] = x.to(bf)
        noise = torch.randn(e - s0, device=dev, generator=g) * 0.02
        v1[s0:e] = (noise if a.far else x + noise * 0.005).to(bf)
    plan = ops.make_slerp_plan(lay.offsets, dev)
    t = torch.full((len(lay),), 0.43, dtype=torch.float64, device=dev)
    st = L.stream_ptr(dev)
    redo = torch.empty(plan.nseg, dtype=torch.int32, device=dev)
    libs = {"intree": lib}
    if a.variants:
        import glob
        for f in sorted(glob.glob(os.path.join(a.variants, "lib*.so"))):
            libs[os.path.basename(f)[3:-3]] = L.load_library(f)

    cases = {"lerp": lambda: lib.edt_lerp(L.ptr(v0), L.ptr(v1), 1, L.ptr(out), 1, 1, P, 0.43, st)}
    # the tensor-list forms (the drop-in path over state-dict tensors) on views of the same arenas
    sizes = [b - a for a, b in zip(lay.offsets, lay.offsets[1:])]
    l0, l1, lo = list(torch.split(v0, sizes)), list(torch.split(v1, sizes)), list(torch.split(out, sizes))
    lplan = ops.make_slerp_plan(lay.offsets, dev, relative=True)
    cases["list_two_pass"] = lambda: ops.slerp_list(lplan, l0, l1, lo, t, speculate=False)
    cases["list_speculative"] = lambda: ops.slerp_list(lplan, l0, l1, lo, t, speculate=True)
    # the same tensors bound once (ops.bind_slerp_list): no per-tensor host work per merge
    bnd = ops.bind_slerp_list(lplan, l0, l1, lo)
    cases["list_bound_two_pass"] = lambda: bnd.merge(t, speculate=False)
    cases["list_bound_speculative"] = lambda: bnd.merge(t, speculate=True)
    for name, lb in libs.items():
        part = torch.empty(int(lb.edt_slerp_sums_doubles(3, plan.nchunks)), dtype=torch.float64, device=dev)

        def spec(lb=lb, part=part):
            return lb.edt_slerp_merge_speculative(
                L.ptr(v0), L.ptr(v1), 1, L.ptr(out), 1, L.ptr(plan.chunks), plan.nchunks, L.ptr(plan.seg_first),
                plan.nseg, L.ptr(t), 0.9995, 1e-8, L.ptr(part), L.ptr(plan.coef), L.ptr(plan.dots),
                L.ptr(redo), P, st)

        def two(lb=lb, part=part):
            return lb.edt_slerp_merge(
                L.ptr(v0), L.ptr(v1), 1, L.ptr(out), 1, L.ptr(plan.chunks), plan.nchunks, L.ptr(plan.seg_first),
                plan.nseg, L.ptr(t), 0.9995, 1e-8, L.ptr(part), L.ptr(plan.coef), L.ptr(plan.dots), st)

        def stats(lb=lb, part=part):
            return lb.edt_slerp_stats(L.ptr(v0), L.ptr(v1), 1, L.ptr(plan.chunks), plan.nchunks, L.ptr(part), st)

        sfx = "" if name == "intree" else f"/{name}"
        cases["speculative" + sfx] = spec
        cases["two_pass" + sfx] = two
        cases["stats" + sfx] = stats
    for k, f in cases.items():
        if not k.startswith("list_"):
            assert f() == 0, L.last_error() if hasattr(L, "last_error") else "launch failed"
        else:
            f()
    torch.cuda.synchronize()
    times = {k: [] for k in cases}
    s = torch.cuda.current_stream(dev)
    for _ in range(a.rounds):
        for k, f in cases.items():
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(s)
            f()
            e1.record(s)
            torch.cuda.synchronize()
            times[k].append(e0.elapsed_time(e1))
    redo_n = int(redo.sum().item())
    # bytes: 6 per element (2 bf16 reads + 1 write); the stats pass reads 4
    res = {k: {"median_ms": round(statistics.median(v), 4), "min_ms": round(min(v), 4),
               "TBps": round((4 if k.startswith("stats") else 6) * P / statistics.median(v) / 1e9, 3)}
           for k, v in times.items()}
    print(json.dumps({"probe": "slerp_spec", "elements": P, "far": a.far, "redo_segments": redo_n,
                      "results": res}))


if __name__ == "__main__":
    main()
