"""Device-resident throughput of the other hot-path kernels (HIP events, one process):

  pair_merge  EDT child (lerp .5 + 2-parent delta + Nesterov SGD), gpt_1p3b, bf16 model + bf16 base
              algorithmic bytes/elem: 4 parents x 2 + child 2 + momentum r/w 4 = 14
  slerp       SLERP crossover of two qwen2p5_7b_body parents (bf16 in, bf16 out), 338 segments
              algorithmic bytes/elem: 2 x 2 in + 2 out = 6 (the 2-pass form reads the parents twice: 10)
  lerp        run_linear_merge_5050 on gpt_1p3b bf16: 2 x 2 in + 2 out = 6
  outer_list  DiLoCo step over SEPARATE tensors (gpt_1p3b: 292 per model, K = 8 bf16 workers, fp32
              theta + momentum; edt_outer_step_list) beside the flat-arena launch on the same data:
              8 x 2 + 4 x 4 = 32 bytes/elem

    python scripts/bench_ops.py [--ops pair,slerp,lerp] [--iters 5]
"""
from __future__ import annotations

import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
PEAK = 8000.0


def timed(fn, iters):
    fn()
    torch.cuda.synchronize()
    out = []
    for _ in range(iters):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        torch.cuda.synchronize()
        out.append(a.elapsed_time(b))
    out.sort()
    return out[len(out) // 2]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ops", default="pair,slerp,lerp,outer_list")
    ap.add_argument("--iters", type=int, default=5)
    ap.add_argument("--slerp-chunks", default="65536",
                    help="comma list of SLERP plan chunk sizes (elements per workgroup chunk) to time")
    ap.add_argument("--list-wdt", default="bf16", choices=["bf16", "f32"], help="outer_list worker dtype")
    a = ap.parse_args()
    from evolutionarydistributedtraining_amd import ops
    from evolutionarydistributedtraining_amd.layouts import gpt_1p3b, qwen2p5_7b_body
    dev = torch.device("cuda:0")
    res = {}
    bf = torch.bfloat16
    if "pair" in a.ops or "lerp" in a.ops:
        P = gpt_1p3b().total
        b1 = (torch.randn(P, device=dev) * 0.02).to(bf)
        b2 = (torch.randn(P, device=dev) * 0.02).to(bf)
        if "pair" in a.ops:
            m1 = (b1.float() + torch.randn(P, device=dev) * 1e-3).to(bf)
            m2 = (b2.float() + torch.randn(P, device=dev) * 1e-3).to(bf)
            out = torch.empty(P, dtype=bf, device=dev)
            mom = (torch.randn(P, device=dev) * 1e-3).to(bf)
            ms = timed(lambda: ops.pair_merge(b1, b2, m1, m2, out, mom, True, 0.7, 0.9, True), a.iters)
            gbs = 14 * P / ms / 1e6
            res["pair_merge"] = {"P": P, "ms": round(ms, 3), "GBps": round(gbs, 1), "frac": round(gbs / PEAK, 4),
                                 "bytes_per_elem": 14}
            del m1, m2, out, mom
        if "lerp" in a.ops:
            out = torch.empty(P, dtype=bf, device=dev)
            ms = timed(lambda: ops.lerp(0.5, b1, b2, out=out), a.iters)
            gbs = 6 * P / ms / 1e6
            res["lerp"] = {"P": P, "ms": round(ms, 3), "GBps": round(gbs, 1), "frac": round(gbs / PEAK, 4),
                           "bytes_per_elem": 6}
        del b1, b2
        torch.cuda.empty_cache()
    if "outer_list" in a.ops:
        lay = gpt_1p3b()
        P, K = lay.total, 8
        theta = torch.randn(P, device=dev) * 0.02
        mom = torch.randn(P, device=dev) * 1e-3
        lw = bf if a.list_wdt == "bf16" else torch.float32
        workers = [(theta + torch.randn(P, device=dev) * 1e-3).to(lw) for _ in range(K)]
        bpe = K * workers[0].element_size() + 16
        ms_flat = timed(lambda: ops.outer_step(theta, workers, mom, True, 0.7, 0.9, True), a.iters)
        th_t = [v.clone() for v in lay.views(theta)]
        mo_t = [v.clone() for v in lay.views(mom)]
        del theta, mom
        w_t = []
        for w in workers:
            w_t.append([v.clone() for v in lay.views(w)])
        del workers, w
        torch.cuda.empty_cache()
        ms = timed(lambda: ops.outer_step_list(th_t, w_t, mo_t, True, 0.7, 0.9, True), a.iters)
        res["outer_list"] = {"P": P, "tensors": len(lay), "K": K, "worker_dtype": a.list_wdt, "ms": round(ms, 3),
                             "GBps": round(bpe * P / ms / 1e6, 1), "frac": round(bpe * P / ms / 1e6 / PEAK, 4),
                             "flat_ms": round(ms_flat, 3), "bytes_per_elem": bpe}
        del th_t, mo_t, w_t
        torch.cuda.empty_cache()
    if "slerp" in a.ops:
        lay = qwen2p5_7b_body()
        P = lay.total
        v0 = torch.empty(P, dtype=bf, device=dev)
        v1 = torch.empty(P, dtype=bf, device=dev)
        out = torch.empty(P, dtype=bf, device=dev)
        chunk_sizes = [int(c) for c in a.slerp_chunks.split(",")]
        plans = {c: ops.make_slerp_plan(lay.offsets, dev, chunk_elems=c) for c in chunk_sizes}
        t = torch.full((len(lay),), 0.5, dtype=torch.float64, device=dev)
        # far: v1 = v0 + 5 % noise (|dot| ~ 0.9988, SLERP branch everywhere);
        # lineage: 0.5 % noise (|dot| ~ 0.99999, the lerp branch: fine-tunes of one base)
        for parents, rel in (("far", 0.05), ("lineage", 0.005)):
            step = 1 << 28
            for s0 in range(0, P, step):
                e = min(P, s0 + step)
                x = torch.randn(e - s0, device=dev) * 0.02
                v0[s0:e] = x.to(bf)
                v1[s0:e] = (x + torch.randn(e - s0, device=dev) * 0.02 * rel).to(bf)
                del x
            for (c, plan), spec in ((cp, sp) for cp in plans.items() for sp in (False, True)):
                ms = timed(lambda: ops.slerp_arena(plan, v0, v1, out, t, speculate=spec), a.iters)
                gbs = 6 * P / ms / 1e6
                tag = "" if len(plans) == 1 else f"/chunk{c}"
                res[f"slerp/{parents}/{'speculative' if spec else 'two_pass'}{tag}"] = {
                    "P": P, "segments": len(lay), "chunks": plan.nchunks, "ms": round(ms, 3),
                    "GBps_algorithmic": round(gbs, 1), "frac": round(gbs / PEAK, 4), "bytes_per_elem": 6,
                    "lerp_branch_segments": int((plan.dots[:len(lay)].abs() > 0.9995).sum().item())}
    print(json.dumps(res))


if __name__ == "__main__":
    main()
