"""The population planner (edt_slerp_population_layout, host only: no GPU needed) on the graphs
EDT_RL's selection draws and on the fallbacks. r5: every component whose distinct dots fit its
slots takes the needed layout (norms + the children's dots: ring dots along the best cyclic order,
the rest chords); the speculative form is member-major for the graphs EDT_RL's selection draws."""
import random

import pytest

from evolutionarydistributedtraining_amd import ops
from evolutionarydistributedtraining_amd.schedule import roulette_generation_pairs


def test_roulette_generations_take_the_needed_layout():
    for g in roulette_generation_pairs(8, 300, seed=17):
        pairs = g["pairs"]
        lay = ops.population_layout(pairs, 8, True)
        assert lay["form"] == "member-major", (pairs, lay)
        D = len({m for p in pairs for m in p})
        assert lay["distinct_parents"] == D
        assert sum(len(c["members"]) for c in lay["components"]) == D
        dots = {tuple(sorted(p)) for p in pairs if p[0] != p[1]}
        assert sum(c["dots"] for c in lay["components"]) == len(dots)
        for c in lay["components"]:
            assert c["stats_layout"] == "needed"
            n = len(c["members"])
            ring = n if n >= 3 else n - 1                 # ring dots (c, c + 1 mod n)
            chords = 0 if n <= 3 else 2 if n == 4 else 4  # chord slots
            assert c["sums"] == n + ring + chords
            assert c["chords"] <= chords and c["picked_pairs"] <= 8
        two = ops.population_layout(pairs, 8, False)
        assert two["form"] == "two-pass" and all(c["stats_layout"] == "needed" for c in two["components"])


def test_selection_statistics_that_motivate_it():
    """The r5 correction: under roulette selection most generations have a parent in >= 3
    distinct pairs (r4's ring layout covers none of them); all are member-major now."""
    hub = 0
    gens = roulette_generation_pairs(8, 2000, seed=3)
    for g in gens:
        deg = {}
        for a, b in {tuple(sorted(p)) for p in g["pairs"]}:
            deg[a] = deg.get(a, 0) + 1
            deg[b] = deg.get(b, 0) + 1
        hub += max(deg.values()) >= 3
    assert hub / len(gens) > 0.5


@pytest.mark.parametrize("pairs,form,layouts", [
    ([(c, (c + 1) % 8) for c in range(8)], "member-major", ["needed"]),
    ([(a, b) for a in range(5) for b in range(a + 1, 5)], "co-located", ["triangle"]),
    ([(m, m + 1) for m in range(8)], "co-located", []),
    ([(0, 1), (1, 0), (0, 2), (2, 0), (1, 2), (2, 1), (0, 3), (3, 0), (1, 3)], "member-major", ["needed"]),
    # 5 members, 4 chords in both orientations + a self-pair: 9 picked pairs > 8 slots
    ([(0, 1), (1, 2), (2, 3), (3, 4), (4, 0), (0, 2), (2, 0), (1, 3), (3, 1), (2, 4), (4, 2), (3, 0), (0, 3),
      (1, 1)], "co-located", ["needed"]),
    ([(3, 6)] * 8, "member-major", ["needed"]),
    ([(4, 4), (2, 2)], "member-major", ["needed", "needed"]),
])
def test_fallbacks(pairs, form, layouts):
    n = max(max(p) for p in pairs) + 1
    lay = ops.population_layout(pairs, n, True)
    assert lay["form"] == form, lay
    assert [c["stats_layout"] for c in lay["components"]] == layouts, lay


def test_layout_rejects_bad_pairs():
    from evolutionarydistributedtraining_amd._lib import EdtError
    with pytest.raises(EdtError):
        ops.population_layout([(0, 9)], 8)


def test_rank_generation_pairs_follow_the_lm_master():
    """schedule.rank_generation_pairs: EDT_LM's rank_based_selection of P - ELITISM distinct
    unordered pairs (two different parents each) + (elite, elite) pairs, deterministic per seed,
    leaving the global random state alone."""
    import random

    from evolutionarydistributedtraining_amd.schedule import rank_generation_pairs
    random.seed(123)
    before = random.getstate()
    gens = rank_generation_pairs(8, 20, seed=9)
    assert random.getstate() == before
    assert gens == rank_generation_pairs(8, 20, seed=9)
    for g in gens:
        pairs = g["pairs"]
        assert len(pairs) == 8 and all(a != b for a, b in pairs)
        assert len({tuple(sorted(p)) for p in pairs}) == 8
    el = rank_generation_pairs(8, 5, seed=9, elitism=2)
    for g in el:
        assert len(g["pairs"]) == 8 and g["pairs"][-1][0] == g["pairs"][-1][1] and g["pairs"][-2][0] == g["pairs"][-2][1]


def test_needed_table_covers_every_child_on_random_graphs():
    """edt_slerp_needed_table on 300 seeded random pair graphs (1..8 members, 1..24 children, self
    pairs, repeats, reversals): every child's two norms and its dot are columns of one block;
    blocks are laid out back to back; a block's columns are its members' norms first; a block on
    the needed layout has D + ring + <= 4 chord slots (triangle otherwise: the norms and the used
    dots formed, the other triangle columns (-1, -1)); the table and scratch
    sizes follow; the planner's JSON view agrees (components, sums per block)."""
    import random

    from evolutionarydistributedtraining_amd import ops
    rng = random.Random(4242)
    for _ in range(300):
        M = rng.randint(1, 8)
        pairs = []
        for _q in range(rng.randint(1, 24)):
            a = rng.randrange(M)
            pairs.append((a, a if rng.random() < 0.1 else rng.randrange(M)))
        nch = rng.randint(1, 500)
        lay = ops.needed_table(pairs, 8, nch)
        cols = {}
        off = 0
        for b, ((o, nt), c) in enumerate(zip(lay.blocks, lay.columns)):
            assert o == off and len(c) == nt
            off += nch * nt
            for x, (i, j) in enumerate(c):
                if i >= 0:
                    cols.setdefault(frozenset((i, j)), set()).add(b)
        assert lay.doubles == off
        for i, j in pairs:
            bi, bj, bd = cols[frozenset((i,))], cols[frozenset((j,))], cols[frozenset((i, j))]
            assert bi & bj & bd, (pairs, i, j)
        js = ops.population_layout(pairs, 8, False)
        assert len(js["components"]) == len(lay.blocks)
        assert [c["sums"] for c in js["components"]] == [nt for _, nt in lay.blocks]
        for comp, c in zip(js["components"], lay.columns):
            D = len(comp["members"])
            if comp["stats_layout"] == "needed":
                assert [set(x) for x in c[:D]] == [{m} for m in comp["members"]]   # norms first
                assert len(c) == 2 * D + (4 if D >= 5 else 2 if D == 4 else 0) - (1 if D <= 2 else 0)
            else:     # the triangle layout (r6: a mode of the needed pass): D(D+1)/2 columns,
                mem = comp["members"]                # the norms and the dots a child uses formed
                assert len(c) == D * (D + 1) // 2
                used = {frozenset((i, j)) for i, j in pairs if i in mem}
                want = sorted([(m, m) for m in mem] + [tuple(sorted(d)) for d in used if len(d) == 2])
                assert sorted(tuple(sorted(x)) for x in c if x[0] >= 0) == want
                assert sum(1 for x in c if x[0] < 0) == len(c) - len(want)
