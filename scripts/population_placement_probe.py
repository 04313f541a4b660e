"""Does the placement of a resident population's OUTPUT arenas move the generation's time, and can a
search recover it (DESIGN §9 open item 3)? The members stay where they are;
the children's arenas are drawn `--draws` times (each draw behind a held spacer, so draws land in
different physical ranges) and the generation is timed on each.

  lm     EDT-LM at 1.3B: 8 members (bf16 base / trained / momentum), the rank-selected pairs of
         generation 0, edt_pair_merge_population; every draw's child arenas stay held (42 GB each)
  slerp  the SLERP population at 7.07B (configs[4]): 8 members, 8 roulette-drawn children of one
         lineage (speculative single pass); one child set (113 GB) at a time, freed between draws
         Then the per-child search: for each child, 3 candidate arenas timed with edt_lerp of its
         two parents into the candidate (the child's own access pattern: its parents read, it
         written), the fastest kept; the generation is timed again on the chosen arenas.

  lm_set the whole EDT-LM set (members and children) drawn in several regions (r6 follow-up)

    python scripts/population_placement_probe.py [lm|lm_set|slerp] > profiles/r06_population_placement.jsonl
"""
import json
import os
import statistics
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from evolutionarydistributedtraining_amd import ops  # noqa: E402
from evolutionarydistributedtraining_amd.layouts import gpt_1p3b, qwen2p5_7b_body  # noqa: E402
from evolutionarydistributedtraining_amd.merge import rl_t_per_segment  # noqa: E402
from evolutionarydistributedtraining_amd.schedule import rank_generation_pairs, roulette_generation_pairs  # noqa: E402

GIB = 1 << 30


def event_ms(fn, n=10, warm=1):
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(n)]
    for a, b in ev:
        a.record()
        fn()
        b.record()
    torch.cuda.synchronize()
    return statistics.median(a.elapsed_time(b) for a, b in ev)


def lm(draws):
    dev = torch.device("cuda:0")
    P, bf, M = gpt_1p3b().total, torch.bfloat16, 8
    g = torch.Generator(device=dev).manual_seed(31)
    x = torch.randn(P, generator=g, device=dev) * 0.02
    base, trained, mom = [], [], []
    for _ in range(M):
        b = (x + torch.randn(P, generator=g, device=dev) * 1e-4).to(bf)
        base.append(b)
        trained.append((b.float() + torch.randn(P, generator=g, device=dev) * 1e-3).to(bf))
        mom.append((torch.randn(P, generator=g, device=dev) * 1e-3).to(bf))
    del x
    pairs = [tuple(p) for p in rank_generation_pairs(M, 1, seed=2025)[0]["pairs"]]
    held, times = [], []
    for d in range(draws):
        if d:
            held.append(torch.empty(d * (11 << 27), dtype=torch.uint8, device=dev))
        outs = [torch.empty(P, dtype=bf, device=dev) for _ in range(M)]
        omom = [torch.empty(P, dtype=bf, device=dev) for _ in range(M)]
        children = [{"b1": base[i], "b2": base[j], "m1": trained[i], "m2": trained[j], "out": outs[c],
                     "momentum": omom[c], "momentum_in": mom[i], "has_momentum": True}
                    for c, (i, j) in enumerate(pairs)]
        ms = event_ms(lambda: ops.pair_merge_population(children, 0.7, 0.9, True))
        times.append(round(ms, 3))
        held.append((outs, omom))
        print(json.dumps({"case": "lm_draw", "draw": d, "ms": round(ms, 3)}), flush=True)
    print(json.dumps({"case": "lm", "P": P, "pairs": [list(p) for p in pairs], "draw_ms": times,
                      "spread": round(max(times) / min(times) - 1, 4)}), flush=True)


def slerp(draws):
    dev = torch.device("cuda:0")
    lay = qwen2p5_7b_body()
    P, bf, M = lay.total, torch.bfloat16, 8
    members = [torch.empty(P, dtype=bf, device=dev) for _ in range(M)]
    g = torch.Generator(device=dev).manual_seed(12)
    for s0 in range(0, P, 1 << 27):
        e = min(P, s0 + (1 << 27))
        x = torch.randn(e - s0, generator=g, device=dev) * 0.02
        for m in members:
            m[s0:e] = (x + torch.randn(e - s0, generator=g, device=dev) * (0.02 * 0.005)).to(bf)
        del x
    plan = ops.make_slerp_plan(lay.offsets, dev)
    t = torch.tensor(rl_t_per_segment(lay.names), dtype=torch.float64, device=dev)
    pairs = [tuple(p) for p in roulette_generation_pairs(M, 1, seed=2025)[0]["pairs"]]
    gen = lambda outs: ops.slerp_population(plan, members, pairs, outs, t, speculate=True)
    times = []
    outs = None
    for d in range(draws):
        outs = None
        torch.cuda.empty_cache()
        spacer = torch.empty(max(1, d * 5 * GIB), dtype=torch.uint8, device=dev) if d else None
        outs = [torch.empty(P, dtype=bf, device=dev) for _ in range(M)]
        ms = event_ms(lambda: gen(outs))
        times.append(round(ms, 3))
        print(json.dumps({"case": "slerp_draw", "draw": d, "ms": round(ms, 3)}), flush=True)
        del spacer
    # per-child search on the last draw: candidates timed with the child's own stream (lerp of its parents)
    search = []
    for c, (i, j) in enumerate(pairs):
        cands = [outs[c]]
        spacers = []
        for k in range(1, 3):
            spacers.append(torch.empty(k * 3 * GIB, dtype=torch.uint8, device=dev))
            cands.append(torch.empty(P, dtype=bf, device=dev))
        tl = [event_ms(lambda o=o: ops.lerp(0.5, members[i], members[j], o), 3, 1) for o in cands]
        best = min(range(len(cands)), key=tl.__getitem__)
        outs[c] = cands[best]
        search.append({"child": c, "lerp_ms": [round(v, 3) for v in tl], "chosen": best})
        del cands, spacers
        torch.cuda.empty_cache()
    placed = event_ms(lambda: gen(outs))
    print(json.dumps({"case": "slerp", "P": P, "pairs": [list(p) for p in pairs], "draw_ms": times,
                      "spread": round(max(times) / min(times) - 1, 4), "last_draw_ms": times[-1],
                      "per_child_search": search, "placed_ms": round(placed, 3)}), flush=True)


def _lm_set(dev, P, M, bf):
    g = torch.Generator(device=dev).manual_seed(31)
    x = torch.randn(P, generator=g, device=dev) * 0.02
    base, trained, mom = [], [], []
    for _ in range(M):
        b = (x + torch.randn(P, generator=g, device=dev) * 1e-4).to(bf)
        base.append(b)
        trained.append((b.float() + torch.randn(P, generator=g, device=dev) * 1e-3).to(bf))
        mom.append((torch.randn(P, generator=g, device=dev) * 1e-3).to(bf))
    del x
    return base, trained, mom


def lm_set(draws):
    """r6 follow-up: the whole EDT-LM set (members' base / trained / momentum and the children's
    arenas) drawn `draws` times, each behind a held spacer of d x 9 GiB with the previous draw
    freed; the same seeded contents every draw (identical work), the generation timed on each."""
    dev = torch.device("cuda:0")
    P, bf, M = gpt_1p3b().total, torch.bfloat16, 8
    pairs = [tuple(p) for p in rank_generation_pairs(M, 1, seed=2025)[0]["pairs"]]
    times = []
    for d in range(draws):
        torch.cuda.empty_cache()
        spacer = torch.empty(d * 9 * GIB, dtype=torch.uint8, device=dev) if d else None
        base, trained, mom = _lm_set(dev, P, M, bf)
        outs = [torch.empty(P, dtype=bf, device=dev) for _ in range(M)]
        omom = [torch.empty(P, dtype=bf, device=dev) for _ in range(M)]
        children = [{"b1": base[i], "b2": base[j], "m1": trained[i], "m2": trained[j], "out": outs[c],
                     "momentum": omom[c], "momentum_in": mom[i], "has_momentum": True}
                    for c, (i, j) in enumerate(pairs)]
        ms = event_ms(lambda: ops.pair_merge_population(children, 0.7, 0.9, True))
        times.append(round(ms, 3))
        print(json.dumps({"case": "lm_set_draw", "draw": d, "ms": round(ms, 3)}), flush=True)
        del children, base, trained, mom, outs, omom, spacer
    print(json.dumps({"case": "lm_set", "P": P, "pairs": [list(p) for p in pairs], "draw_ms": times,
                      "spread": round(max(times) / min(times) - 1, 4)}), flush=True)


if __name__ == "__main__":
    which = sys.argv[1] if len(sys.argv) > 1 else "lm"
    {"lm": lambda: lm(int(os.environ.get("DRAWS", "4"))),
     "lm_set": lambda: lm_set(int(os.environ.get("DRAWS", "4"))),
     "slerp": lambda: slerp(int(os.environ.get("DRAWS", "3")))}[which]()
