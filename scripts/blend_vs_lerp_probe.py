"""Is the far-parent SLERP blend slower than lerp's identical stream (2 bf16 reads + 1 bf16
write per element), or is the gap the arena size? Times, in one process on the same arenas:
edt_lerp over the flat 7B body, edt_slerp_blend over the same arenas (chunk-table tiles, per-segment
coefficients), and both over the first 1.3B elements. HIP events, median of interleaved rounds.

    python scripts/blend_vs_lerp_probe.py [--rounds 8]
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
    ap.add_argument("--rounds", type=int, default=8)
    a = ap.parse_args()
    from evolutionarydistributedtraining_amd import _lib as L
    from evolutionarydistributedtraining_amd import ops
    from evolutionarydistributedtraining_amd.layouts import gpt_1p3b, qwen2p5_7b_body
    dev = torch.device("cuda:0")
    lib = L.lib()
    big = qwen2p5_7b_body()
    P = big.total
    bf = torch.bfloat16
    v0 = torch.empty(P, dtype=bf, device=dev)
    v1 = torch.empty(P, dtype=bf, device=dev)
    out = torch.empty(P, dtype=bf, device=dev)
    for s0 in range(0, P, 1 << 28):
        e = min(P, s0 + (1 << 28))
        x = torch.randn(e - s0, device=dev) * 0.02
        v0[s0:e] = x.to(bf)
        v1[s0:e] = (x + torch.randn(e - s0, device=dev) * 1e-3).to(bf)
    small_n = gpt_1p3b().total
    plans = {"7b": (ops.make_slerp_plan(big.offsets, dev), P),
             "1p3b": (ops.make_slerp_plan([o for o in big.offsets if o <= small_n], dev), None)}
    st = L.stream_ptr(dev)
    cases = {}
    for key, (plan, _) in plans.items():
        n = plan.seg_offsets[-1]
        plan.coef.fill_(0.5)
        cases[f"lerp/{key}"] = (n, lambda n=n: lib.edt_lerp(L.ptr(v0), L.ptr(v1), 1, L.ptr(out), 1, 1, n, 0.5, st))
        cases[f"blend/{key}"] = (n, lambda plan=plan: lib.edt_slerp_blend(
            L.ptr(v0), L.ptr(v1), 1, L.ptr(out), 1, L.ptr(plan.chunks), plan.nchunks, L.ptr(plan.coef), st))
    for _, f in cases.values():
        assert f() == 0
    torch.cuda.synchronize()
    times = {k: [] for k in cases}
    for _ in range(a.rounds):
        for k, (_, f) in cases.items():
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            f()
            e1.record()
            torch.cuda.synchronize()
            times[k].append(e0.elapsed_time(e1))
    res = {k: {"elements": cases[k][0], "median_ms": round(statistics.median(v), 4),
               "TBps": round(6 * cases[k][0] / statistics.median(v) / 1e9, 3)} for k, v in times.items()}
    print(json.dumps({"probe": "blend_vs_lerp", "results": res}, indent=1))


if __name__ == "__main__":
    main()
