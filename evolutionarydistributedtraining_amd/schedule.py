"""Selection -> exchange schedule.

The reference's masters pick parent pairs with Python's global `random` module, then ship model
directories between machines. The selection functions below restate theirs draw for draw (same
`random` calls in the same order, so a seeded master picks the same pairs), and
`exchange_plan` turns a selection into the point-to-point transfers that bring every child's
parents to the GPU that builds it (one population member per GPU, RCCL send/recv over xGMI —
each GPU has a direct link to every other, so a plan is a set of independent link transfers).

  rank_based_selection      EDT_LM/edt_sim.py:177-214, EDT_LM/edt.py:185-211, EDT_EVOMERGE/edt.py:193-230
  tournament_selection      EDT_LM/edt.py:213-224
  spin_roulette / roulette_wheel_selection   EDT_RL/edt.py:221-240
  rank_based_selection_rl   EDT_RL/edt.py:243-261
  roulette_scale            EDT_RL/edt.py:264-265
"""
from __future__ import annotations

import random

YELLOW, RESET = "\033[33m", "\033[0m"


def rank_based_selection(genomes, num_pairs):
    """Linear-rank selection of distinct, not-yet-used pairs (1000 attempts, then any distinct pair)."""
    ranked = sorted(genomes, key=lambda g: g["fitness"], reverse=True)
    n = len(ranked)
    weights = [(2 * (n - i)) / (n * (n + 1)) for i in range(n)]
    seen, pairs = set(), []
    for _ in range(num_pairs):
        for _attempt in range(1000):
            a = random.choices(ranked, weights=weights, k=1)[0]
            b = random.choices(ranked, weights=weights, k=1)[0]
            key = tuple(sorted([a["model_path"], b["model_path"]]))
            if a != b and key not in seen:
                seen.add(key)
                pairs.append((a, b))
                break
        else:
            print(f"{YELLOW}Warning: Could not find unique pair after 1000 attempts{RESET}")
            while True:
                a = random.choices(ranked, weights=weights, k=1)[0]
                b = random.choices(ranked, weights=weights, k=1)[0]
                if a != b:
                    pairs.append((a, b))
                    break
    return pairs


def tournament_selection(genomes, num_pairs, tournament_size=3):
    """Each parent is the fittest of a random sample; the two parents must differ."""
    pairs = []
    k = min(tournament_size, len(genomes))
    for _ in range(num_pairs):
        while True:
            a = max(random.sample(genomes, k), key=lambda g: g["fitness"])
            b = max(random.sample(genomes, k), key=lambda g: g["fitness"])
            if a != b:
                pairs.append((a, b))
                break
    return pairs


def spin_roulette(genomes, sum_fitness, scale):
    pick = random.random() * sum_fitness
    running = 0
    for g in genomes:
        running += g["fitness"] ** scale
        if running >= pick:
            return g
    return genomes[-1]


def roulette_wheel_selection(genomes, num_pairs, scale):
    """Fitness-proportional (fitness ** scale) pairs of distinct parents."""
    total = sum(g["fitness"] ** scale for g in genomes)
    pairs = []
    for _ in range(num_pairs):
        a = spin_roulette(genomes, total, scale)
        b = spin_roulette(genomes, total, scale)
        while b == a:
            b = spin_roulette(genomes, total, scale)
        pairs.append((a, b))
    return pairs


def rank_based_selection_rl(genomes, num_pairs):
    """The RL master's rank selection: weight rank/sum(ranks) over the fitness-sorted list."""
    ranked = sorted(genomes, key=lambda g: g["fitness"], reverse=True)
    ranks = list(range(1, len(ranked) + 1))
    total = sum(ranks)
    weights = [r / total for r in ranks]
    pairs = []
    for _ in range(num_pairs):
        a = random.choices(ranked, weights=weights, k=1)[0]
        b = random.choices(ranked, weights=weights, k=1)[0]
        while b == a:
            b = random.choices(ranked, weights=weights, k=1)[0]
        pairs.append((a, b))
    return pairs


def roulette_scale(generation_index, max_generations):
    return 0.1 + 2.4 * min(generation_index / max_generations, 1.0)


def pair_indices(pairs, genomes, key="model_path"):
    """Selected genome pairs -> (i, j) member indices in `genomes`."""
    where = {g[key]: i for i, g in enumerate(genomes)}
    return [(where[a[key]], where[b[key]]) for a, b in pairs]


def exchange_plan(pairs, owner, child_rank):
    """Point-to-point transfers that deliver every child's parents to the rank that builds it.

    pairs[c] = (i, j): parents of child c (member indices); owner[m]: rank holding member m;
    child_rank[c]: rank building child c. Returns {rank: {"send": [(member, dst)],
    "recv": [(member, src)]}}, one transfer per (member, destination) however many children on
    that destination use it; nothing is sent to a rank that already holds the member."""
    ranks = set(owner) | set(child_rank)
    plan = {r: {"send": [], "recv": []} for r in ranks}
    done = set()
    for c, (i, j) in enumerate(pairs):
        dst = child_rank[c]
        for m in (i, j):
            src = owner[m]
            if src == dst or (m, dst) in done:
                continue
            done.add((m, dst))
            plan[src]["send"].append((m, dst))
            plan[dst]["recv"].append((m, src))
    return plan


def link_bytes(plan, member_bytes):
    """Bytes over each directed xGMI link (src, dst) for a plan."""
    out = {}
    for src, p in plan.items():
        for m, dst in p["send"]:
            out[(src, dst)] = out.get((src, dst), 0) + member_bytes
    return out


def roulette_generation_pairs(n_members: int, generations: int, seed: int = 0,
                              scales=(0.1, 1.0, 2.5), num_pairs: int | None = None):
    """Pair graphs as the RL master draws them, for benches and tests: per generation, random
    fitness for `n_members` genomes, then EDT_RL/edt.py:268-269's roulette_wheel_selection of
    n = len(all_genomes) pairs (distinct parents per pair, sampled with replacement across pairs) at
    a scale from `scales` (roulette_scale spans 0.1 .. 2.5 over a run), as member indices. Returns
    [{"source": "roulette", "scale", "seed", "pairs"}]. A private random.Random drives the same
    draws the master's global `random` makes (the functions above call the module's `random`, so
    its state is saved and restored around each draw)."""
    out = []
    rng = random.Random(seed)
    k = num_pairs if num_pairs is not None else n_members
    for g in range(generations):
        scale = scales[g % len(scales)]
        genomes = [{"fitness": rng.uniform(0.05, 1.0), "model_path": f"m{m}"} for m in range(n_members)]
        state = random.getstate()
        random.seed(rng.getrandbits(64))
        try:
            pairs = pair_indices(roulette_wheel_selection(genomes, k, scale), genomes)
        finally:
            random.setstate(state)
        out.append({"source": "roulette", "scale": scale, "seed": seed, "generation": g, "pairs": pairs})
    return out


def rank_generation_pairs(n_members: int, generations: int, seed: int = 0, elitism: int = 0):
    """Pair graphs as the EDT-LM master draws them (EDT_LM/edt_sim.py:215-243, EDT_LM/edt.py:226-260):
    per generation, random fitness for `n_members` genomes, rank_based_selection of
    n_members - elitism distinct pairs, then (elite, elite) for the top `elitism` genomes, as
    member indices. Same private-RNG discipline as roulette_generation_pairs."""
    out = []
    rng = random.Random(seed)
    for g in range(generations):
        genomes = [{"fitness": rng.uniform(0.05, 1.0), "model_path": f"m{m}"} for m in range(n_members)]
        state = random.getstate()
        random.seed(rng.getrandbits(64))
        try:
            sel = rank_based_selection(genomes, n_members - elitism) if n_members > 1 else [(genomes[0], genomes[0])]
        finally:
            random.setstate(state)
        ranked = sorted(genomes, key=lambda x: x["fitness"], reverse=True)
        sel += [(e, e) for e in ranked[:elitism]] if n_members > 1 else []
        out.append({"source": "rank", "elitism": elitism, "seed": seed, "generation": g,
                    "pairs": pair_indices(sel, genomes)})
    return out
