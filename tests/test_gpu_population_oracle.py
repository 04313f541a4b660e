"""The resident SLERP population against the reference restatement directly (Weak 1:
test_gpu_population_needed.py holds each child to the HIP pair merge, which is pinned to the
reference only through test_gpu_refdot.py / test_gpu_slerp_order.py; here the population's own
outputs are held to the oracle, on the pair graphs the reference's selection draws).

EDT_RL/edt.py:231-240, 268-269 (roulette_wheel_selection, 8 pairs with replacement) ->
EDT_RL/edt.py:286-299 -> EDT_RL/crossover.py:11-43 per child and per state-dict key:
  * reference-dot mode (ops.RefDot): every child, every tensor, both branches, both forms
    (speculative needed-sums pass / two-pass) equals oracle.slerp_parts_refdot — the reference's
    SLERP restated on the pinned host — BIT FOR BIT;
  * default (fp64 dot): every tensor the oracle puts in the lerp branch, and the device too, is
    bit-exact with oracle.slerp_parts; the SLERP-branch tensors are within the golden bar (the
    oracle's dot is fp32, the device's fp64: DESIGN.md §3).
"""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

SIZES = [70001, 33, 131072, 5, 8192 * 3 + 7, 1, 65536, 12289]


@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    return torch.device("cuda:0")


def _graphs():
    from evolutionarydistributedtraining_amd.schedule import roulette_generation_pairs
    g = {f"roulette_{k}": [tuple(p) for p in gd["pairs"]]
         for k, gd in enumerate(roulette_generation_pairs(8, 4, seed=2025))}
    g["k5_dense"] = [(a, b) for a in range(5) for b in range(a + 1, 5)]
    g["star16"] = [(0, m) for m in range(1, 8)] + [(m, 0) for m in range(1, 8)] + [(2, 3), (3, 2)]
    return g


GRAPHS = _graphs()


def _members(dev, dt, seed=7):
    """8 members: lineage ones (lerp branch on most tensors) and far ones (SLERP branch)."""
    from evolutionarydistributedtraining_amd.params import ParamLayout
    layout = ParamLayout([(n,) for n in SIZES])
    g = torch.Generator().manual_seed(seed)
    base = torch.randn(layout.total, generator=g) * 0.02
    mem = [(base + torch.randn(layout.total, generator=g) * 0.02 * [0.002, 0.01, 1.0][m % 3]).to(dt)
           for m in range(8)]
    return layout, mem


def _run(dev, layout, mem, pairs, out_dt, speculate, ref):
    from evolutionarydistributedtraining_amd import ops
    plan = ops.make_slerp_plan(layout.offsets, dev)
    t = torch.tensor([0.5, 0.3, 0.7, 0.0, 1.0, 0.43333333333333335, 0.9, 0.5][:len(SIZES)], dtype=torch.float64,
                     device=dev)
    outs = [torch.full((layout.total,), float("nan"), dtype=out_dt, device=dev) for _ in pairs]
    ops.slerp_population(plan, [m.to(dev) for m in mem], pairs, outs, t, speculate=speculate,
                         ref_dot=ops.RefDot() if ref else None)
    torch.cuda.synchronize()
    return [o.cpu() for o in outs], t.cpu().tolist()


@pytest.mark.parametrize("speculate", [True, False])
@pytest.mark.parametrize("name", sorted(GRAPHS))
def test_population_refdot_equals_reference_restatement(oracle, dev, name, speculate):
    layout, mem = _members(dev, torch.bfloat16)
    pairs = GRAPHS[name]
    outs, t = _run(dev, layout, mem, pairs, torch.float32, speculate, ref=True)
    offs = layout.offsets
    cache, branches = {}, set()
    for q, (i, j) in enumerate(pairs):
        for s in range(len(SIZES)):
            a, b = offs[s], offs[s + 1]
            key = (i, j, s)
            if key not in cache:
                want, _, lerp = oracle.slerp_parts_refdot(t[s], mem[i][a:b], mem[j][a:b])
                cache[key] = (torch.from_numpy(np.ascontiguousarray(np.ravel(want)).astype(np.float32)), lerp)
            want, lerp = cache[key]
            branches.add(lerp)
            assert torch.equal(outs[q][a:b].view(torch.int32), want.view(torch.int32)), (name, speculate, q, i, j, s)
    assert True in branches


@pytest.mark.parametrize("name", ["roulette_0", "roulette_3", "k5_dense"])
def test_population_default_mode_lerp_branch_exact(oracle, dev, name):
    """The fp64-dot default: the lerp branch is bit-exact with the reference restatement; the
    SLERP branch within the golden bar |out - ref| <= 2e-6 (|c0 v0| + |c1 v1|) + 1.01 |dc| |v|."""
    layout, mem = _members(dev, torch.float32, seed=11)
    pairs = GRAPHS[name]
    offs = layout.offsets
    for speculate in (True, False):
        outs, t = _run(dev, layout, mem, pairs, torch.float32, speculate, ref=False)
        n_lerp = 0
        for q, (i, j) in enumerate(pairs):
            for s in range(len(SIZES)):
                a, b = offs[s], offs[s + 1]
                v0, v1 = mem[i][a:b], mem[j][a:b]
                want, dot, lerp = oracle.slerp_parts(t[s], v0, v1)
                want = torch.from_numpy(np.ascontiguousarray(np.ravel(want)).astype(np.float32))
                got = outs[q][a:b]
                if lerp and abs(float(dot)) > 0.9995 + 1e-5:          # both dots clearly in the lerp branch
                    n_lerp += 1
                    assert torch.equal(got.view(torch.int32), want.view(torch.int32)), (name, q, s)
                elif not lerp:
                    # the SLERP branch: the oracle's fp32 dot and the device's fp64 one differ by
                    # < 1e-5 here; the coefficients move by at most the formula's change over that
                    # (plus its rounding noise, tests/test_gpu_fuzz.py::_coef_allowance)
                    from tests.test_gpu_fuzz import _coef_allowance
                    c0, c1, _ = oracle.slerp_coefficients(t[s], v0, v1)
                    d0, d1 = _coef_allowance(oracle, t[s], float(dot), 1e-5)
                    bar = 1.01 * (d0 * v0.abs() + d1 * v1.abs()) \
                        + 2e-6 * (abs(float(c0)) * v0.abs() + abs(float(c1)) * v1.abs()) + 1e-12
                    assert bool(((got - want).abs() <= bar).all()), (name, q, s, float((got - want).abs().max()))
        assert n_lerp > 0
