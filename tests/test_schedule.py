"""Selection -> exchange schedule: the restated selection functions draw exactly what the
reference's masters draw (golden pairs recorded from their source), and the exchange plan
delivers every parent exactly once per destination."""
import random

import pytest

from evolutionarydistributedtraining_amd import schedule

FNS = {
    "rank_based_lm_sim": schedule.rank_based_selection,
    "rank_based_lm": schedule.rank_based_selection,
    "rank_based_evomerge": schedule.rank_based_selection,
    "tournament_lm": schedule.tournament_selection,
    "roulette_rl": schedule.roulette_wheel_selection,
    "rank_based_rl": schedule.rank_based_selection_rl,
}


def test_selection_matches_reference_draws(golden):
    sel = golden.manifest["selection"]
    genomes = sel["genomes"]
    assert len(sel["cases"]) == 72
    for c in sel["cases"]:
        random.seed(c["seed"])
        args = (genomes, c["num_pairs"]) + ((c["scale"],) if "scale" in c else ())
        pairs = FNS[c["fn"]](*args)
        got = [[genomes.index(a), genomes.index(b)] for a, b in pairs]
        assert got == c["pairs"], c


def test_roulette_scale():
    assert schedule.roulette_scale(0, 10) == pytest.approx(0.1)
    assert schedule.roulette_scale(10, 10) == pytest.approx(2.5)
    assert schedule.roulette_scale(20, 10) == pytest.approx(2.5)


def test_exchange_plan_delivers_each_parent_once():
    random.seed(5)
    genomes = [{"model_path": f"m{i}", "fitness": 0.1 + i / 10} for i in range(8)]
    pairs = schedule.pair_indices(schedule.rank_based_selection(genomes, 8), genomes)
    owner = list(range(8))                    # member m lives on GPU m
    child_rank = list(range(8))               # child c is built on GPU c
    plan = schedule.exchange_plan(pairs, owner, child_rank)
    # every child's parents are local or received, each (member, dst) transferred once
    for c, (i, j) in enumerate(pairs):
        have = {m for m, _ in plan[c]["recv"]} | {m for m in range(8) if owner[m] == c}
        assert i in have and j in have
    sends = [(m, d) for r in plan for m, d in plan[r]["send"]]
    assert len(sends) == len(set(sends))
    recvs = sorted((m, r) for r in plan for m, _ in plan[r]["recv"])
    assert recvs == sorted(sends)
    assert all(owner[m] == r for r in plan for m, _ in plan[r]["send"])
    lb = schedule.link_bytes(plan, 14_000_000_000)
    assert all(src != dst for src, dst in lb)


def test_exchange_plan_self_pair_needs_no_transfer():
    plan = schedule.exchange_plan([(0, 0), (1, 1)], [0, 1], [0, 1])
    assert plan == {0: {"send": [], "recv": []}, 1: {"send": [], "recv": []}}
