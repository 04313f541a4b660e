"""One EDT generation's data path with the population resident in HBM (population.py,
SURVEY.md §8(f) row 4), on one GPU: selection -> (no exchange at world 1) -> P child merges ->
swap. Compare: the reference moves each child through the shared disk (crossover.py loads four
checkpoints and saves one; profiles/r01_crossover_e2e.json: 0.24 s per 162M child with the
direct arena reader, 3.7 s through from_pretrained).

  sgd    EDT-LM children (edt_pair_merge_population: all children in one launch, a parent's
         chunk read from HBM once for all its children), bf16 members + bf16 outer momentum, steady
         state. Per child and element (children independent): 4 parents x 2 +
         child 2 + donor momentum read 2 + child momentum write 2 = 14 B. The generation's floor:
         every distinct parent's base and trained weights (+ momentum if a donor) once, every
         child and its momentum once.
  slerp  EDT-RL / EVOMERGE children, per-tensor t, bf16 in / bf16 out: 2 x 2 in + 2 out = 6 B per
         child; edt_slerp_population runs one Gram stats pass over the members and one
         co-located blend launch for all children, so its floor is two reads of every distinct
         parent + one write per child.

    python scripts/bench_generation.py [--layout gpt2_small] [--population 8] [--iters 5]
"""
from __future__ import annotations

import argparse
import json
import os
import random
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
PEAK_TBPS = 8.0


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--layout", default="gpt2_small")
    ap.add_argument("--population", type=int, default=8)
    ap.add_argument("--kinds", default="sgd,slerp")
    ap.add_argument("--iters", type=int, default=5)
    ap.add_argument("--json", default=None)
    ap.add_argument("--slerp-chunk", type=int, default=None, help="SLERP plan chunk (elements per workgroup)")
    ap.add_argument("--members", default="lineage", choices=["lineage", "random"],
                    help="lineage: one base + 0.5 %% per-member noise (fine-tunes of a common base: the "
                         "SLERP takes the lerp branch); random: independent members (SLERP branch)")
    a = ap.parse_args()
    from evolutionarydistributedtraining_amd.layouts import LAYOUTS
    from evolutionarydistributedtraining_amd.merge import merge_plan
    from evolutionarydistributedtraining_amd.population import ResidentPopulation
    dev = torch.device("cuda:0")
    layout = LAYOUTS[a.layout]()
    n, P = layout.total, a.population
    out = {"layout": a.layout, "params": n, "population": P, "members": a.members, "results": {}}
    for kind in a.kinds.split(","):
        random.seed(0)
        if kind == "sgd":
            genomes = [{"dna": [m % 4, (m + 1) % 4, (m + 2) % 4]} for m in range(P)]
            pop = ResidentPopulation(layout, torch.bfloat16, dev, genomes, kind="sgd", elitism=1)
            arenas = [pop.base(m) for m in range(P)] + [pop.trained(m) for m in range(P)]
        else:
            genomes = [{"env": {"env_name": "e", "reward_dna": [m] * 6, "agents": []}} for m in range(P)]
            t = [t for _, t in merge_plan(layout.names, 24, {"parameters": {"t": [
                {"filter": "self_attn", "value": [0, .5, .3, .7, 1]}, {"filter": "mlp", "value": [1, .5, .7, .3, 0]},
                {"value": 0.5}]}})]
            if len(t) != len(layout):
                t = [0.5] * len(layout)
            pop = ResidentPopulation(layout, torch.bfloat16, dev, genomes, kind="slerp", seg_t=t,
                                     slerp_chunk=a.slerp_chunk)
            arenas = [pop.params(m) for m in range(P)]
        g = torch.Generator(device=dev).manual_seed(1)
        step = 1 << 28                      # fill in chunks: fp32 temporaries stay ~1 GiB at 7B
        for s0 in range(0, n, step):
            e = min(n, s0 + step)
            common = torch.randn(e - s0, generator=g, device=dev) * 0.02 if a.members == "lineage" else None
            for x in arenas:
                if common is None:
                    x[s0:e].copy_(torch.randn(e - s0, generator=g, device=dev) * 0.02)
                else:
                    x[s0:e].copy_(common + torch.randn(e - s0, generator=g, device=dev) * 0.02 * 0.005)
            del common
        fitness = [float(m) for m in range(P)]
        pop.step(fitness)                      # generation 0 (first-step momentum), warm-up
        torch.cuda.synchronize()
        times, host, used = [], [], None
        for _ in range(a.iters):
            h0 = time.perf_counter()
            pairs = pop.select(fitness)
            host.append(time.perf_counter() - h0)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            pop.crossover(pairs)
            e1.record()
            torch.cuda.synchronize()
            times.append(e0.elapsed_time(e1))
            used = pairs
        times.sort()
        ms = times[len(times) // 2]
        # SURVEY 8(d) accounting, children independent: 14 B (sgd) / 6 B (slerp) per child and element
        per_child = 14 if kind == "sgd" else 6
        survey = per_child * n * P
        # the generation's floor: every distinct parent array read once (per pass), every output once
        parents = sorted({m for pr in used for m in pr})
        donors = {i for i, _ in used}                     # steady state: parent 1 carries momentum
        if kind == "sgd":
            floor = n * (len(parents) * 2 * 2 + len(donors) * 2 + P * 2 * 2)
        else:
            # two passes (Gram + blend) or, speculative, one pass + a second over the SLERP-branch
            # share f of the elements: the cheaper of the two (the form ops picks)
            import numpy as np
            d = pop._plan._pop_dots.cpu().numpy()
            sizes = np.diff(np.asarray(layout.offsets, dtype=np.int64))
            f = float((sizes[None, :] * (np.abs(d) <= 0.9995)).sum()) / (int(sizes.sum()) * d.shape[0])
            one = n * (len(parents) * 2 + P * 2)
            floor = int(min(2 * n * len(parents) * 2 + n * P * 2, (1 + f) * one))
        out["results"][kind] = {
            "generation_ms": round(ms, 3), "per_child_ms": round(ms / P, 4),
            "survey_bytes": survey, "survey_TBps": round(survey / ms / 1e9, 3),
            "floor_bytes": floor, "floor_TBps": round(floor / ms / 1e9, 3),
            "frac_of_8TBps_at_floor": round(floor / ms / 1e9 / PEAK_TBPS, 4),
            "distinct_parents": len(parents),
            "host_select_ms": round(1e3 * sorted(host)[len(host) // 2], 3),
        }
        print(kind, out["results"][kind], flush=True)
        del pop, arenas
        torch.cuda.empty_cache()
    print(json.dumps(out))
    if a.json:
        with open(a.json, "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
