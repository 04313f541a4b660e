"""Probe: does the two-pass SLERP's second read of the parents come from the 256 MiB Infinity
Cache when the merge runs over groups of whole tensors instead of the whole 7B arena at once?
(the far-parent form moves 10 B per 6 algorithmic; a blend pass that re-reads
parents still resident on-die would move ~6 B of HBM traffic.)

For each group size, the 7B body's tensors are packed into groups of whole tensors (a tensor's dot
needs all of it) and `ops.slerp_arena(..., speculate=False)` runs once per group, back to back on
one stream; the time is HIP events around the whole sweep; the child must equal the whole-arena
child bit for bit.

    python scripts/slerp_mall_probe.py [--groups 0,256,128,64,32] (MiB of both parents per group; 0 = whole)
        [--variants shipped,s_nt0,s_rev,s_rev_nt0]   (libraries from scripts/kernel_variants.py --build)
"""
from __future__ import annotations

import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from evolutionarydistributedtraining_amd import ops
    from evolutionarydistributedtraining_amd.layouts import qwen2p5_7b_body
    ap = argparse.ArgumentParser()
    ap.add_argument("--groups", default="0,512,256,192,128,64,32")
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--variants", default="")
    a = ap.parse_args()
    from evolutionarydistributedtraining_amd import _lib as L
    vdir = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "build_variants")
    variants = [("" if v == "shipped" else v) for v in a.variants.split(",")] if a.variants else [""]
    dev = torch.device("cuda:0")
    lay = qwen2p5_7b_body()
    P, bf = lay.total, torch.bfloat16
    g = torch.Generator(device=dev).manual_seed(3)
    v0 = torch.empty(P, dtype=bf, device=dev)
    v1 = torch.empty(P, dtype=bf, device=dev)
    step = 1 << 28
    for s in range(0, P, step):
        e = min(P, s + step)
        x = torch.randn(e - s, generator=g, device=dev) * 0.02
        v0[s:e] = x.to(bf)
        v1[s:e] = (x + torch.randn(e - s, generator=g, device=dev) * 0.02).to(bf)   # far parents
    out = torch.empty(P, dtype=bf, device=dev)
    ref = torch.empty(P, dtype=bf, device=dev)
    offs = lay.offsets
    t_all = torch.full((len(lay),), 0.5, dtype=torch.float64, device=dev)
    plan = ops.make_slerp_plan(offs, dev)
    L.load_library()
    shipped = L._lib
    ops.slerp_arena(plan, v0, v1, ref, t_all, speculate=False)
    torch.cuda.synchronize()
    sizes = [offs[i + 1] - offs[i] for i in range(len(offs) - 1)]
    big = max(sizes)
    res = {"layout": "qwen2p5_7b_body", "P": P, "tensors": len(sizes), "largest_tensor_MiB_both": big * 4 / 2**20,
           "algo_bytes": 6 * P, "runs": []}
    cases = [(v, int(x)) for v in variants for x in a.groups.split(",")]
    for var, gmib in cases:
        L._lib = L.load_library(os.path.join(vdir, var + ".so")) if var else shipped
        if gmib == 0:
            groups = [(0, len(sizes))]
        else:
            groups, g0 = [], 0
            for i in range(1, len(sizes)):          # tensor i joins [g0, i) unless that overflows
                if (offs[i + 1] - offs[g0]) * 4 > gmib * 2**20:
                    groups.append((g0, i))
                    g0 = i
            groups.append((g0, len(sizes)))
        gplans = [ops.make_slerp_plan([o - offs[s] for o in offs[s:e + 1]], dev) for s, e in groups]

        def run():
            for (s, e), gp in zip(groups, gplans):
                a0, a1 = offs[s], offs[e]
                ops.slerp_arena(gp, v0[a0:a1], v1[a0:a1], out[a0:a1], t_all[s:e], speculate=False)

        out.zero_()
        run()
        torch.cuda.synchronize()
        same = bool(torch.equal(out.view(torch.int16), ref.view(torch.int16)))
        ts = []
        for _ in range(a.reps):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            run()
            e1.record()
            torch.cuda.synchronize()
            ts.append(e0.elapsed_time(e1))
        ms = min(ts)
        res["runs"].append({"variant": var or "shipped", "group_MiB": gmib, "groups": len(groups), "launch_sets": len(groups), "ms": round(ms, 3),
                            "algo_TBps": round(6 * P / ms / 1e9, 3), "frac": round(6 * P / ms / 1e9 / 8.0, 3),
                            "equal_whole_arena": same})
        print(json.dumps(res["runs"][-1]), file=sys.stderr, flush=True)
        del gplans
    L._lib = shipped
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
