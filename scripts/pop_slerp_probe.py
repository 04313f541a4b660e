"""BASELINE configs[4] on one MI355X, timed warm: a resident population of 8 Qwen2.5-7B bodies (bf16)
SLERP-crossed into 8 children (edt_slerp_population*), in each kernel form:
lineage members and independent members, each through both forms (ops.slerp_population with
speculate=True: one co-located pass + SLERP-branch redo; False: the Gram stats pass + member-major
blends) — `--rounds` generations after one warm-up each, HIP events around each generation.
Run under rocprofv3 --kernel-trace --stats for the per-kernel split.

    python scripts/pop_slerp_probe.py [--rounds 3]
"""
import argparse
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
BF = torch.bfloat16


def fill(dst, gen, scale, base=None, rel=0.0):
    step = 1 << 28
    for s in range(0, dst.numel(), step):
        e = min(dst.numel(), s + step)
        x = torch.randn(e - s, device=dst.device, generator=gen) * scale
        if base is not None:
            x = base[s:e].float() + x * rel
        dst[s:e] = x.to(dst.dtype)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--variants", default="", help="also run every lib*.so in DIR (build_slerp_variants.py)")
    ap.add_argument("--pairs", default="probe", choices=("probe", "ring"),
                    help="probe: ((3c+1) % 8, (5c+2) % 8), a matching with every pair twice; ring: (c, c+1 % 8), "
                         "the bench's ring of children")
    a = ap.parse_args()
    from evolutionarydistributedtraining_amd import _lib as L
    from evolutionarydistributedtraining_amd import ops
    from evolutionarydistributedtraining_amd.layouts import qwen2p5_7b_body
    dev = torch.device("cuda:0")
    lay = qwen2p5_7b_body()
    P, N = lay.total, 8
    gen = torch.Generator(device=dev).manual_seed(4)
    members = [torch.empty(P, dtype=BF, device=dev) for _ in range(N)]
    outs = [torch.empty(P, dtype=BF, device=dev) for _ in range(N)]
    t = torch.rand(len(lay), dtype=torch.float64, generator=torch.Generator().manual_seed(4)).to(dev)
    plan = ops.make_slerp_plan(lay.offsets, dev)
    pairs = ([((3 * c + 1) % N, (5 * c + 2) % N) for c in range(N)] if a.pairs == "probe"
             else [(c, (c + 1) % N) for c in range(N)])
    s = torch.cuda.current_stream(dev)
    res, sigs = {}, {}

    def run(name, speculate):
        ts = []
        for r in range(a.rounds + 1):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(s)
            dots = ops.slerp_population(plan, members, pairs, outs, t, speculate=speculate)
            e1.record(s)
            torch.cuda.synchronize()
            if r:
                ts.append(e0.elapsed_time(e1))
        slerp_share = float((dots.abs() <= 0.9995).float().mean())
        # the dots (every Gram / pair sum feeds them) and a strided sample of every child, against
        # the first build's same form on the same members: a variant must give the same bits
        sig = torch.cat([dots.reshape(-1).view(torch.int64).double(),
                         torch.stack([o[::7919].view(torch.int16).double().sum() for o in outs])])
        key = name.split("/")[0]
        same = None
        if key in sigs:
            same = bool(torch.equal(sigs[key], sig))
        else:
            sigs[key] = sig
        res[name] = {"median_ms": round(statistics.median(ts), 3), "min_ms": round(min(ts), 3),
                     "children": N, "distinct_parents": len({m for p in pairs for m in p}),
                     "slerp_branch_segment_share": round(slerp_share, 3),
                     "GBps_algorithmic": round(2 * P * (len({m for p in pairs for m in p}) + N)
                                               / statistics.median(ts) / 1e6, 1)}
        if same is not None:
            res[name]["bit_identical_to_first_build"] = same
        print(name, res[name], flush=True)

    base = torch.empty(P, dtype=BF, device=dev)
    fill(base, gen, 0.02)
    for m in members:
        fill(m, gen, 0.02, base=base, rel=0.005)       # one lineage: every segment in the lerp branch
    del base
    import glob
    libs = [("", L.load_library())] + [("/" + os.path.basename(f)[3:-3], L.load_library(f))
                                       for f in sorted(glob.glob(os.path.join(a.variants, "lib*.so")))] \
        if a.variants else [("", L.load_library())]
    intree = L._lib

    def forms(tag):
        for sfx, lb in libs:
            L._lib = lb                                # ops.* call through L.lib(): this build
            run(f"{tag}_speculative{sfx}", True)
            run(f"{tag}_gram_two_pass{sfx}", False)
        L._lib = intree

    forms("lineage")
    for m in members:
        fill(m, gen, 0.02)                             # independent members: the SLERP branch
    forms("independent")
    print(json.dumps({"probe": "pop_slerp", "pairs": a.pairs, "elements_per_member": P, "results": res}))


if __name__ == "__main__":
    main()
