"""The EDT-LM generation (edt_pair_merge_population) on rank-selected pair graphs at 1.3B, bf16:
the in-tree build against variant libraries (`--variants DIR`: every lib*.so there, e.g. built with
variant tunables; r5 compared the member-major forms since removed), interleaved rounds, HIP-event medians; every variant's children and momenta
compared bit for bit with the in-tree build's.

    python scripts/lm_population_probe.py [--variants variants] [--generations 3] [--rounds 3]
"""
import argparse
import glob
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--variants", default="")
    ap.add_argument("--generations", type=int, default=3)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--layout", default="gpt_1p3b")
    a = ap.parse_args()
    from evolutionarydistributedtraining_amd import _lib as L
    from evolutionarydistributedtraining_amd import ops
    from evolutionarydistributedtraining_amd.layouts import LAYOUTS
    from evolutionarydistributedtraining_amd.schedule import rank_generation_pairs
    dev = torch.device("cuda:0")
    P, bf, M = LAYOUTS[a.layout]().total, torch.bfloat16, 8
    g = torch.Generator(device=dev).manual_seed(31)
    x = torch.randn(P, generator=g, device=dev) * 0.02
    base, trained, mom = [], [], []
    for m in range(M):
        b = (x + torch.randn(P, generator=g, device=dev) * 1e-4).to(bf)
        base.append(b)
        trained.append((b.float() + torch.randn(P, generator=g, device=dev) * 1e-3).to(bf))
        mom.append((torch.randn(P, generator=g, device=dev) * 1e-3).to(bf))
    del x
    outs = [torch.empty(P, dtype=bf, device=dev) for _ in range(M)]
    omom = [torch.empty(P, dtype=bf, device=dev) for _ in range(M)]
    libs = [("in-tree", L.load_library())]
    if a.variants:
        libs += [(os.path.basename(f), L.load_library(f)) for f in sorted(glob.glob(os.path.join(a.variants, "lib*.so")))]
    intree = L._lib
    gens = [[tuple(p) for p in gd["pairs"]] for gd in rank_generation_pairs(M, a.generations, seed=2025)]

    def children(pairs):
        return [{"b1": base[i], "b2": base[j], "m1": trained[i], "m2": trained[j], "out": outs[c], "momentum": omom[c],
                 "momentum_in": mom[i], "has_momentum": True} for c, (i, j) in enumerate(pairs)]

    def timed(fn, n=10):
        fn()
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(n)]
        for s, e in ev:
            s.record()
            fn()
            e.record()
        torch.cuda.synchronize()
        return statistics.median(s.elapsed_time(e) for s, e in ev)

    want = {}
    L._lib = intree
    for k, pairs in enumerate(gens):
        ops.pair_merge_population(children(pairs), 0.7, 0.9, True)
        torch.cuda.synchronize()
        want[k] = [(o.clone(), m.clone()) for o, m in zip(outs, omom)]
    res, same = {}, {}
    for r in range(a.rounds):
        for name, lib in libs:
            L._lib = lib
            for k, pairs in enumerate(gens):
                ch = children(pairs)
                res.setdefault(f"{name}/gen{k}", []).append(round(timed(lambda: ops.pair_merge_population(ch, 0.7, 0.9, True)), 4))
                if r == 0:
                    torch.cuda.synchronize()
                    same[f"{name}/gen{k}"] = all(torch.equal(o.view(torch.int16), w[0].view(torch.int16)) and
                                                 torch.equal(m.view(torch.int16), w[1].view(torch.int16))
                                                 for o, m, w in zip(outs, omom, want[k]))
        L._lib = intree
        print(json.dumps({k: v[-1] for k, v in res.items()}), flush=True)
    floors = {k: P * (4 * len({x for p in pairs for x in p}) + 2 * len({i for i, _ in pairs}) + 4 * len(pairs))
              for k, pairs in enumerate(gens)}
    out = {k: {"median_ms": statistics.median(v), "floor_TBps": round(floors[int(k.split("gen")[1])] /
                                                                         (statistics.median(v) / 1e3) / 1e12, 3),
               "bit_identical": same.get(k)} for k, v in res.items()}
    print(json.dumps({"probe": "lm_population", "pairs": gens, "results": out}))


if __name__ == "__main__":
    main()
