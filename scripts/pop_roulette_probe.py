"""BASELINE configs[4] on one MI355X on the pair graphs the reference's own selection draws: a
resident population of 8 Qwen2.5-7B bodies (bf16) SLERP-crossed into 8 children per generation,
the parents drawn by EDT_RL/edt.py:231-240's roulette_wheel_selection (schedule.py, the same
`random` draws; n = 8 pairs, scale 0.1 / 1.0 / 2.5 as roulette_scale spans it, random fitness) and
t per key from EDT_RL/crossover.py:146-147's layer curves (merge.t_for_key, 28 layers).

Per drawn graph: both forms of ops.slerp_population (speculative single pass, two-pass) on lineage
members, `--rounds` timed calls after one warm-up, HIP events; the graph's distinct parents,
components and the layout each component took (ops.population_layout). `--ring` adds the ring of
children (c, c + 1 mod 8) as a labelled reference case.

    python scripts/pop_roulette_probe.py [--graphs 6] [--rounds 3] [--ring] [--independent]
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
    ap.add_argument("--graphs", type=int, default=6)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--seed", type=int, default=2025)
    ap.add_argument("--ring", action="store_true")
    ap.add_argument("--independent", action="store_true", help="also independent members (SLERP branch)")
    ap.add_argument("--out", default="")
    ap.add_argument("--only", type=int, default=-1, help="run only graph k of the drawn list (-1: all)")
    ap.add_argument("--forms", default="speculative,two_pass")
    a = ap.parse_args()
    from evolutionarydistributedtraining_amd import ops
    from evolutionarydistributedtraining_amd.layouts import qwen2p5_7b_body
    from evolutionarydistributedtraining_amd.merge import rl_t_per_segment
    from evolutionarydistributedtraining_amd.schedule import roulette_generation_pairs
    dev = torch.device("cuda:0")
    lay = qwen2p5_7b_body()
    P, N = lay.total, 8
    gen = torch.Generator(device=dev).manual_seed(4)
    members = [torch.empty(P, dtype=BF, device=dev) for _ in range(N)]
    outs = [torch.empty(P, dtype=BF, device=dev) for _ in range(N)]
    t = torch.tensor(rl_t_per_segment(lay.names), dtype=torch.float64, device=dev)
    plan = ops.make_slerp_plan(lay.offsets, dev)
    graphs = roulette_generation_pairs(N, a.graphs, seed=a.seed)
    if a.ring:
        graphs.append({"source": "ring", "scale": None, "pairs": [(c, (c + 1) % N) for c in range(N)]})
    if a.only >= 0:
        graphs = [graphs[a.only]]
    s = torch.cuda.current_stream(dev)
    res = []

    def run(g, kind):
        pairs = [tuple(p) for p in g["pairs"]]
        D = len({m for p in pairs for m in p})
        rec = {"members": kind, "source": g["source"], "scale": g["scale"], "pairs": pairs, "distinct_parents": D,
               "layout": ops.population_layout(pairs, N)}
        for form, spec, floor in (("speculative", True, 2 * P * (D + N)), ("two_pass", False, 2 * P * (2 * D + N))):
            if form not in a.forms.split(","):
                continue
            ts = []
            for r in range(a.rounds + 1):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(s)
                ops.slerp_population(plan, members, pairs, outs, t, speculate=spec)
                e1.record(s)
                torch.cuda.synchronize()
                if r:
                    ts.append(e0.elapsed_time(e1))
            ms = statistics.median(ts)
            rec[form] = {"median_ms": round(ms, 3), "min_ms": round(min(ts), 3), "floor_bytes": floor,
                         "floor_GBps": round(floor / ms / 1e6, 1)}
        print(json.dumps(rec), flush=True)
        res.append(rec)

    base = torch.empty(P, dtype=BF, device=dev)
    fill(base, gen, 0.02)
    for m in members:
        fill(m, gen, 0.02, base=base, rel=0.005)       # one lineage: every segment in the lerp branch
    del base
    for g in graphs:
        run(g, "lineage")
    if a.independent:
        for m in members:
            fill(m, gen, 0.02)
        for g in graphs:
            run(g, "independent")
    out = {"probe": "pop_roulette", "elements_per_member": P, "results": res}
    if a.out:
        with open(a.out, "w") as f:
            json.dump(out, f, indent=1)
    print(json.dumps({"summary": [(r["members"], r["distinct_parents"], r.get("speculative", {}).get("median_ms"),
                                   r.get("two_pass", {}).get("median_ms")) for r in res]}))


if __name__ == "__main__":
    main()
