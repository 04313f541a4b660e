"""The needed-sums population passes (r5) on the pair graphs the reference's selection draws.

EDT_RL/edt.py:231-240, 268-269 draws n = 8 pairs by roulette with replacement: most generations
have a parent in >= 3 pairs, which neither r4's ring layout nor a fixed layout covers. Every
component of the pair graph now forms only its members' norms and the dots its children use, and
the speculative form writes every child's lerp-branch output from the same registers. Bar: every
child's output and per-segment dot bit-identical to edt_slerp_merge on its two parents (whose
sums are pinned to the canonical order by test_gpu_slerp_order.py), in both forms — roulette
draws at the three scales roulette_scale spans, dense graphs past the dot slots (triangle /
co-located fallbacks), duplicate children (one output computed, stored to each), reversed pairs,
every child on one pair, and the fp32 dtype routes.
"""
import pytest
import torch

from tests.golden_data import bits

pytestmark = pytest.mark.gpu

SIZES = [0, 1, 7, 33, 4096, 70_001, 0, 129, 200_003, 12_289]


@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    return torch.device("cuda:0")


@pytest.fixture(scope="module")
def ops():
    from evolutionarydistributedtraining_amd import ops as o
    return o


def _roulette(n):
    from evolutionarydistributedtraining_amd.schedule import roulette_generation_pairs
    return [g["pairs"] for g in roulette_generation_pairs(8, n, seed=505)]


ROULETTE = _roulette(24)
EDGE_CASES = {
    "k5_dense": [(a, b) for a in range(5) for b in range(a + 1, 5)],                 # 10 dots > 8 slots
    "all_on_one_pair": [(3, 6)] * 8,
    "pair_and_reverse": [(1, 2), (2, 1), (1, 2), (2, 1), (5, 0), (0, 5), (7, 7), (4, 4)],
    "star16": [(0, m) for m in range(1, 8)] + [(m, 0) for m in range(1, 8)] + [(2, 3), (3, 2)],
    "k4_both_ways": [(0, 1), (1, 0), (0, 2), (2, 0), (1, 2), (2, 1), (0, 3), (3, 0), (1, 3)],
    "emit_overflow": [(0, 1), (1, 2), (2, 3), (3, 4), (4, 0), (0, 2), (2, 0), (1, 3), (3, 1), (2, 4), (4, 2),
                      (3, 0), (0, 3), (1, 1)],                                    # 9 picked pairs > 8
    "nine_parents": [(m, m + 1) for m in range(8)],
}


def _population(dev, nmem, in_dt, seed):
    g = torch.Generator().manual_seed(seed)
    offs = [0]
    for x in SIZES:
        offs.append(offs[-1] + x)
    base = torch.randn(offs[-1], generator=g) * 0.02
    # odd members one lineage step from the base (lerp branch), even ones farther (SLERP branch)
    mem = [(base + torch.randn(offs[-1], generator=g) * (1e-5 if m % 2 else 1e-3)).to(in_dt).to(dev)
           for m in range(nmem)]
    ts = torch.tensor([0.5, 0.0, 1.0, 0.43333333333333335, 0.5, 0.7, 0.5, 0.2, 0.9, 0.3],
                      dtype=torch.float64).to(dev)
    return offs, mem, ts


def _check(ops, dev, pairs, speculate, in_dt=torch.bfloat16, out_dt=torch.bfloat16, seed=0):
    nmem = max(max(p) for p in pairs) + 1
    offs, mem, ts = _population(dev, nmem, in_dt, seed)
    plan = ops.make_slerp_plan(offs, dev, chunk_elems=4096)
    outs = [torch.full((offs[-1],), float("nan"), dtype=out_dt, device=dev) for _ in pairs]
    dots = ops.slerp_population(plan, mem, pairs, outs, ts, speculate=speculate).clone()
    for q, (i, j) in enumerate(pairs):
        want = torch.empty(offs[-1], dtype=out_dt, device=dev)
        ops.slerp_arena(plan, mem[i], mem[j], want, ts, speculate=False)
        assert torch.equal(bits(outs[q].cpu()), bits(want.cpu())), (pairs, speculate, q, i, j)
        assert torch.equal(dots[q].cpu(), plan.dots[:len(SIZES)].cpu()), (pairs, speculate, q, i, j)


@pytest.mark.parametrize("speculate", [False, True])
@pytest.mark.parametrize("k", range(len(ROULETTE)))
def test_roulette_drawn_generations(dev, ops, k, speculate):
    pairs = ROULETTE[k]
    lay = ops.population_layout(pairs, 8, speculate)
    assert all(c["stats_layout"] == "needed" for c in lay["components"]), lay
    if speculate:
        assert lay["form"] == "member-major", lay
    _check(ops, dev, pairs, speculate, seed=k)


@pytest.mark.parametrize("speculate", [False, True])
@pytest.mark.parametrize("case", sorted(EDGE_CASES))
def test_needed_layout_edge_cases(dev, ops, case, speculate):
    if case == "nine_parents" and not speculate:     # the two-pass form takes <= 8 members
        from evolutionarydistributedtraining_amd._lib import EdtError
        with pytest.raises(EdtError):
            _check(ops, dev, EDGE_CASES[case], speculate)
        return
    _check(ops, dev, EDGE_CASES[case], speculate, seed=len(case))


@pytest.mark.parametrize("in_dt,out_dt", [(torch.float32, torch.float32), (torch.bfloat16, torch.float32),
                                          (torch.float32, torch.bfloat16)])
@pytest.mark.parametrize("k", [0, 5])
def test_roulette_drawn_dtype_routes(dev, ops, k, in_dt, out_dt):
    for speculate in (False, True):
        _check(ops, dev, ROULETTE[k], speculate, in_dt=in_dt, out_dt=out_dt, seed=100 + k)


def _random_graphs(n, seed=77):
    import random
    rng = random.Random(seed)
    out = []
    for _ in range(n):
        M = rng.randint(1, 8)
        Q = rng.randint(1, 24)
        pairs = []
        for _q in range(Q):
            a = rng.randrange(M)
            b = a if rng.random() < 0.1 else rng.randrange(M)        # self pairs, repeats, reversals
            pairs.append((a, b))
        out.append(pairs)
    return out


RANDOM_GRAPHS = _random_graphs(40)


@pytest.mark.parametrize("k", range(len(RANDOM_GRAPHS)))
def test_random_pair_graphs_both_forms(dev, ops, k):
    """Seeded random pair graphs over 1..8 members with 1..24 children (self pairs, repeated and
    reversed pairs, isolated members, components of every size; the planner picks needed / triangle
    / member-major / co-located per case): both forms bit-identical to edt_slerp_merge per child."""
    pairs = RANDOM_GRAPHS[k]
    for speculate in (False, True):
        _check(ops, dev, pairs, speculate, seed=300 + k)
