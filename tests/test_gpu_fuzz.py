"""Differential fuzzing of the HIP kernels against the oracle (hypothesis): random sizes (odd,
tiny, vector-boundary), populations, dtype regimes and — what the fixed-parameter tests do not
vary — arbitrary outer-optimiser scalars (lr, momentum, Nesterov, first step or carried buffer) and
lerp weights. The scalars are where the reference's conversions bite: torch rounds `alpha` to
bf16 for bf16 tensors, `mul_(s)` keeps the fp32 scalar, `/ K` is a true division, so a
kernel that folded or rounded a scalar differently would show up here on some draw. Every case is
bit-exact. Reference: EDT_LM/diloco.py:238-289, EDT_LM/train/crossover.py:50-51,150-237."""
import numpy as np
import pytest
import torch
from hypothesis import HealthCheck, given, settings
from hypothesis import strategies as st

from tests.golden_data import bits

pytestmark = pytest.mark.gpu

REGIMES = [(torch.float32, torch.float32), (torch.float32, torch.bfloat16), (torch.bfloat16, torch.bfloat16)]
FUZZ = settings(max_examples=200, deadline=None, derandomize=True,
                suppress_health_check=[HealthCheck.function_scoped_fixture, HealthCheck.too_slow])

sizes = st.one_of(st.integers(1, 40), st.integers(1, 5000), st.sampled_from([7, 8, 9, 2047, 2048, 2049, 4097]))
scalars = st.floats(min_value=1e-4, max_value=2.0, allow_nan=False, allow_infinity=False)


@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.skip("needs a HIP device")
    return torch.device("cuda:0")


@FUZZ
@given(n=sizes, K=st.integers(1, 12), regime=st.sampled_from(REGIMES), lr=scalars,
       mu=st.one_of(st.just(0.0), st.floats(0.0, 0.999)), nesterov=st.booleans(), has=st.booleans(),
       seed=st.integers(0, 2**31 - 1))
def test_outer_step_fuzz(oracle, dev, n, K, regime, lr, mu, nesterov, has, seed):
    from evolutionarydistributedtraining_amd import ops
    gdt, wdt = regime
    if nesterov and mu == 0:
        nesterov = False                     # torch.optim.SGD rejects Nesterov without momentum
    g = torch.Generator().manual_seed(seed)
    theta = (torch.randn(n, generator=g) * 0.02).to(gdt)
    workers = [(theta.float() + torch.randn(n, generator=g) * 1e-3).to(wdt) for _ in range(K)]
    mom = (torch.randn(n, generator=g) * 1e-3).to(gdt)
    th_d, m_d = theta.to(dev), mom.to(dev)
    ops.outer_step(th_d, [w.to(dev) for w in workers], m_d if mu else None, has, lr, mu, nesterov)
    oracle.outer_step(theta, workers, mom if mu else None, has, lr, mu, nesterov)
    assert torch.equal(bits(th_d.cpu()), bits(theta))
    if mu:
        assert torch.equal(bits(m_d.cpu()), bits(mom))


@FUZZ
@given(n=sizes, lr=scalars, mu=st.one_of(st.just(0.0), st.floats(0.0, 0.999)), nesterov=st.booleans(),
       has=st.booleans(), regime=st.sampled_from([(torch.bfloat16, torch.bfloat16), (torch.float32, torch.float32),
                                                  (torch.float32, torch.bfloat16)]),
       seed=st.integers(0, 2**31 - 1))
def test_pair_merge_fuzz(oracle, dev, n, lr, mu, nesterov, has, regime, seed):
    from evolutionarydistributedtraining_amd import ops
    gdt, wdt = regime
    if nesterov and mu == 0:
        nesterov = False
    g = torch.Generator().manual_seed(seed)
    b1, b2 = [(torch.randn(n, generator=g) * 0.02).to(wdt) for _ in range(2)]
    m1 = (b1.float() + torch.randn(n, generator=g) * 1e-3).to(wdt)
    m2 = (b2.float() + torch.randn(n, generator=g) * 1e-3).to(wdt)
    mom = (torch.randn(n, generator=g) * 1e-3).to(gdt)
    out_d = torch.empty(n, dtype=gdt, device=dev)
    mom_d = mom.to(dev)
    ops.pair_merge(b1.to(dev), b2.to(dev), m1.to(dev), m2.to(dev), out_d, mom_d if mu else None, has, lr, mu,
                   nesterov)
    out = torch.empty(n, dtype=gdt)
    oracle.pair_merge(b1, b2, m1, m2, out, mom if mu else None, has, lr, mu, nesterov)
    assert torch.equal(bits(out_d.cpu()), bits(out))
    if mu:
        assert torch.equal(bits(mom_d.cpu()), bits(mom))


@FUZZ
@given(n=sizes, t=st.floats(0.0, 1.0), dt=st.sampled_from([torch.float32, torch.bfloat16]),
       seed=st.integers(0, 2**31 - 1))
def test_lerp_fuzz(oracle, dev, n, t, dt, seed):
    from evolutionarydistributedtraining_amd import ops
    g = torch.Generator().manual_seed(seed)
    v0, v1 = [(torch.randn(n, generator=g) * 0.02).to(dt) for _ in range(2)]
    got = ops.lerp(t, v0.to(dev), v1.to(dev))
    want = oracle.lerp(t, v0, v1)
    assert torch.equal(bits(got.cpu()), bits(want))


@FUZZ
@given(sizes_=st.lists(st.integers(0, 3000), min_size=1, max_size=5),
       ts=st.lists(st.floats(0.0, 1.0), min_size=5, max_size=5),
       spread=st.sampled_from([1e-4, 0.01, 0.05, 0.5, 2.0]), seed=st.integers(0, 2**31 - 1),
       speculate=st.booleans(), layout=st.sampled_from(["arena", "list"]), ref=st.booleans())
def test_slerp_fuzz(oracle, dev, sizes_, ts, spread, seed, speculate, layout, ref):
    """Multi-tensor SLERP (EDT_RL/crossover.py:11-43) over random segment sizes (empty included),
    per-segment t and parent distances from lineage (lerp branch) to far (SLERP branch), both
    kernel forms, over flat arenas or separate tensors (the tensor-list path).
    ref=True (reference-dot mode, ops.RefDot): every segment, both branches, BIT-EXACT with the
    reference restated on the pinned host (oracle.slerp_parts_refdot: its BLAS / numpy dot, numpy's
    float32 coefficients and blend).
    ref=False (the fp64-dot default): per segment the branch agrees with the oracle's (fp32) dot
    away from the threshold, the lerp branch is bit-exact, the SLERP branch is within the golden
    bar; and the device's coefficients are the reference formula at the device's OWN dot within a
    fixed multiple of the formula's conditioning (_coef_strict: no dot uncertainty in it)."""
    from evolutionarydistributedtraining_amd import ops
    g = torch.Generator().manual_seed(seed)
    offs = [0]
    for s in sizes_:
        offs.append(offs[-1] + s)
    n = offs[-1]
    v0 = torch.randn(n, generator=g) * 0.02
    v1 = v0 + torch.randn(n, generator=g) * 0.02 * spread
    t = torch.tensor(ts[:len(sizes_)], dtype=torch.float64)
    ce = 8192 if ref else 1024              # the reference-dot mode's chunks: whole numpy buffers
    rd = ops.RefDot() if ref else None
    if layout == "arena":
        plan = ops.make_slerp_plan(offs, dev, chunk_elems=ce)
        out_d = torch.empty(max(n, 1), dtype=torch.float32, device=dev)[:n]
        ops.slerp_arena(plan, v0.to(dev), v1.to(dev), out_d, t.to(dev), speculate=speculate, ref_dot=rd)
        got = out_d.cpu()
    else:
        plan = ops.make_slerp_plan(offs, dev, chunk_elems=ce, relative=True)
        pieces = list(zip(offs, offs[1:]))
        outs = [torch.empty(b - a, dtype=torch.float32, device=dev) for a, b in pieces]
        ops.slerp_list(plan, [v0[a:b].to(dev) for a, b in pieces], [v1[a:b].to(dev) for a, b in pieces], outs,
                       t.to(dev), speculate=speculate, ref_dot=rd)
        got = torch.cat([o.cpu() for o in outs])
    coef, dots = plan.coef.cpu(), plan.dots.cpu()
    for s in range(len(sizes_)):
        a, b = offs[s], offs[s + 1]
        if b == a:
            continue
        if ref:
            want, wdot, _ = oracle.slerp_parts_refdot(float(t[s]), v0[a:b], v1[a:b])
            assert float(dots[s]) == float(wdot), s
            assert torch.equal(bits(got[a:b]), bits(torch.from_numpy(np.ascontiguousarray(np.ravel(want))))), s
            continue
        _coef_strict(float(t[s]), float(dots[s]), float(coef[s, 0]), float(coef[s, 1]))
        want = oracle.slerp(float(t[s]), v0[a:b], v1[a:b]).float()
        c0, c1, dot = oracle.slerp_coefficients(float(t[s]), v0[a:b], v1[a:b])
        if abs(abs(float(dot)) - 0.9995) < 1e-5:
            continue                                     # the threshold contract's own tests
        err = (got[a:b] - want).abs()
        if abs(float(dot)) > 0.9995:
            assert torch.equal(bits(got[a:b]), bits(want)), s
            continue
        # SLERP branch: our dot (fp64 sums) is within the fp32 dot's error of the reference's, and
        # our coefficients are the reference's formula within its own conditioning at that dot
        # uncertainty (t near 0 or 1: th0 - th0 * t cancels, so a one-ulp move of th0 moves c0
        # by ~1e-5 relative); the output is then bounded by the coefficient gap plus rounding.
        g0, g1 = float(coef[s, 0]), float(coef[s, 1])
        ddot = abs(float(dots[s]) - float(dot))
        assert ddot <= 2e-6, (s, ddot)
        allow = _coef_allowance(oracle, float(t[s]), float(dot), ddot)
        assert abs(g0 - float(c0)) <= allow[0] and abs(g1 - float(c1)) <= allow[1], (s, g0, c0, g1, c1, allow)
        tol = _tol(c0, c1, v0[a:b], v1[a:b]) + 1.01 * (abs(g0 - float(c0)) * v0[a:b].abs()
                                                         + abs(g1 - float(c1)) * v1[a:b].abs())
        assert (err <= tol).all(), (s, err.max().item())


def _coef_strict(t, dot, g0, g1):
    """The device's (c0, c1) against the reference formula in numpy float32 at the device's own
    dot: no dot uncertainty, only the two implementations' transcendental rounding, so
    the bar is a fixed number of ulps scaled by the formula's conditioning A (a 1-ulp move of th0
    moves the result by ~A ulps: th0 (|cot th0| + (1 - t)|cot(th0 - th_t)| + t |cot th_t|), and
    t / (1 - t) from th0 - th_t's cancellation). Host model of correctly rounded fp32 transcendentals
    against numpy's stays under 1.8 (1 + A) ulps over 600k draws; the bar is 6 (1 + A). t > 0.99
    (cancellation beyond the model) and the lerp branch are skipped."""
    import numpy as np
    f = np.float32
    if abs(dot) > 0.9995 or t > 0.99:
        return
    r0, r1 = (float(x) for x in np.asarray(_np_coef(t, dot), dtype=np.float32))
    th0 = float(np.arccos(f(dot)))
    tht = th0 * t
    cot = lambda x: abs(np.cos(x) / np.sin(x)) if abs(np.sin(x)) > 1e-30 else 0.0
    A = th0 * (cot(th0) + (1 - t) * cot(th0 - tht) + t * cot(tht)) + t / (1 - t)
    bar = 6 * (1 + A)
    for g, r in ((g0, r0), (g1, r1)):
        ulp = float(np.spacing(f(abs(r)))) if r != 0 else float(np.spacing(f(0)))
        assert abs(g - r) <= bar * ulp + 1e-38, (t, dot, g, r, abs(g - r) / ulp, bar)


def _np_coef(t, dot):
    from evolutionarydistributedtraining_amd.ops import reference_coefficients
    import numpy as np
    return reference_coefficients(np.float32([dot]), np.float64([t]))[0]


def _tol(c0, c1, v0, v1):
    return 2e-6 * (abs(float(c0)) * v0.float().abs() + abs(float(c1)) * v1.float().abs()) + 1e-30


def _coef_allowance(oracle, t, dot, ddot):
    """How far two evaluations of the reference's own fp32 formula (EDT_RL/crossover.py:36-43) may
    put (c0, c1) apart when their dots differ by ddot: the formula's smooth change over dot +- d
    (d = ddot + a few ulps, for arccos / sin implementations an ulp or two apart), plus its
    ROUNDING NOISE — th_t = th0 * t is rounded, and th0 - th_t cancels for t near 1 (th_t itself is
    small for t near 0), so c0 carries a relative error of up to ulp(th_t) / (th0 - th_t) and c1 one
    of ulp(th_t) / th_t, whatever th0's exact bits: two implementations whose th0 differ by one ulp
    land on unrelated roundings — plus 4 ulps of each coefficient."""
    import numpy as np
    f = np.float32
    th0 = f(np.arccos(f(dot)))
    tht = f(th0 * f(t))
    d = ddot + 4 * float(np.spacing(th0)) * max(float(np.sin(th0)), 1e-30) + 2 * float(np.spacing(f(dot)))
    r0, r1 = oracle.slerp_coefficients_at_dot(t, dot)
    out = [0.0, 0.0]
    for x in (dot - d, dot + d):
        c = oracle.slerp_coefficients_at_dot(t, min(max(x, -1.0), 1.0), dot_threshold=2.0)
        out[0] = max(out[0], abs(float(c[0]) - float(r0)))
        out[1] = max(out[1], abs(float(c[1]) - float(r1)))
    rnd = 4 * (float(np.spacing(tht)) + float(np.spacing(th0)))
    noise0 = abs(float(r0)) * rnd / max(float(th0 - tht), 1e-30)
    noise1 = abs(float(r1)) * rnd / max(float(tht), 1e-30)
    return (out[0] + noise0 + 4 * float(np.spacing(f(abs(r0)))), out[1] + noise1 + 4 * float(np.spacing(f(abs(r1)))))


@settings(max_examples=30, deadline=None, derandomize=True,
          suppress_health_check=[HealthCheck.function_scoped_fixture, HealthCheck.too_slow])
@given(world=st.integers(1, 8), k_local=st.integers(1, 3),
       shapes=st.lists(st.one_of(st.tuples(st.integers(1, 5000)), st.tuples(st.integers(1, 70), st.integers(1, 70))),
                       min_size=1, max_size=6),
       units=st.integers(1, 9), mode=st.sampled_from(["exact", "reduce_ordered"]), workers_bcast=st.booleans(),
       dts=st.sampled_from(REGIMES))
def test_sharded_schedules_fuzz_on_virtual_ranks(dev, world, k_local, shapes, units, mode, workers_bcast, dts):
    """The HIP kernels inside the sharded schedules on random virtual worlds, layouts and bucket
    sizes: exact (either broadcast) bit-exact with the fused single-GPU step over the whole
    population; reduce_ordered bit-exact with per-rank edt_delta_partial + edt_sgd_apply_sum."""
    from evolutionarydistributedtraining_amd import ops
    from tests.virtual_schedules import population, run_sharded
    tdt, wdt = dts
    broadcast = "workers" if workers_bcast and mode == "exact" else "theta"
    k_total = k_local * world
    layout, theta, gens = population(shapes, tdt, wdt, k_total, steps=2, seed=world * 7 + units, device=dev)
    res = run_sharded(world, layout, tdt, wdt, theta, gens, dev, mode=mode, broadcast=broadcast,
                      bucket_elems=units * world * 64)
    n = layout.total
    th, mom = theta.clone(), torch.zeros(n, dtype=tdt, device=dev)
    for i, ws in enumerate(gens):
        if mode == "exact":
            ops.outer_step(th, ws, mom, i > 0, 0.7, 0.9, True)
        else:
            accs = []
            for r in range(world):
                acc = torch.empty(n, device=dev)
                ops.delta_partial(th, ws[r * k_local:(r + 1) * k_local], k_total, acc, False)
                accs.append(acc)
            ops.sgd_apply_sum(th, accs, mom, i > 0, 0.7, 0.9, True)
    torch.cuda.synchronize()
    for r in res:
        assert torch.equal(bits(r["theta"][:n].cpu()), bits(th.cpu())), r
    assert torch.equal(bits(res[0]["mom"].cpu()), bits(mom.cpu()))
    if broadcast == "workers":
        for r in res:
            for w in r["workers"]:
                assert torch.equal(bits(w[:n].cpu()), bits(th.to(wdt).cpu()))


@settings(max_examples=25, deadline=None, derandomize=True,
          suppress_health_check=[HealthCheck.function_scoped_fixture, HealthCheck.too_slow])
@given(world=st.integers(1, 8), groups=st.integers(1, 4),
       shapes=st.lists(st.one_of(st.tuples(st.integers(1, 20000)), st.tuples(st.integers(1, 90), st.integers(1, 90))),
                       min_size=1, max_size=7),
       seed=st.integers(0, 2**31 - 1), roulette=st.booleans())
def test_sharded_population_fuzz_on_virtual_ranks(dev, world, groups, shapes, seed, roulette):
    """The link-balanced population crossover with the HIP needed-sums / coefficient / blend passes
    on random layouts (1,024-element chunks: many chunks per rank, ranges starting off the vector
    grid), worlds, pipeline groups and pair graphs (a fixed permutation-like graph, or r5: drawn by
    EDT_RL's roulette selection): every child bit-identical to edt_slerp_merge on its two parents
    with the same chunk table."""
    from evolutionarydistributedtraining_amd import ops
    from evolutionarydistributedtraining_amd.collectives import VirtualWorld
    from evolutionarydistributedtraining_amd.distributed import ShardedPopulationCrossover
    from evolutionarydistributedtraining_amd.params import ParamLayout
    layout = ParamLayout(shapes)
    n = layout.total
    g = torch.Generator().manual_seed(seed)
    base = torch.randn(n, generator=g) * 0.02
    members = [(base + torch.randn(n, generator=g) * 0.02 * (0.005 if r % 2 else 0.1)).bfloat16().to(dev)
               for r in range(world)]
    pairs = [((3 * c + 1) % world, (5 * c + 2) % world) for c in range(world)]
    if roulette and world > 1:
        from evolutionarydistributedtraining_amd.schedule import roulette_generation_pairs
        pairs = [tuple(p) for p in roulette_generation_pairs(world, 1, seed=seed)[0]["pairs"]]
    t = torch.rand(len(shapes), generator=g, dtype=torch.float64).to(dev)

    def body(comm):
        sp = ShardedPopulationCrossover(layout, torch.bfloat16, dev, comm=comm, chunk_elems=1024, groups=groups)
        out = torch.empty(n, dtype=torch.bfloat16, device=dev)
        sp.slerp_step(members[comm.rank], pairs, t, out)
        torch.cuda.synchronize()
        return out

    res = VirtualWorld(world).run(body)
    plan = ops.make_slerp_plan(layout.offsets, dev, chunk_elems=1024)
    want = torch.empty(n, dtype=torch.bfloat16, device=dev)
    for c, (i, j) in enumerate(pairs):
        ops.slerp_arena(plan, members[i], members[j], want, t, speculate=False)
        torch.cuda.synchronize()
        assert torch.equal(res[c].view(torch.int16), want.view(torch.int16)), c


@settings(max_examples=200, deadline=None, derandomize=True,
          suppress_health_check=[HealthCheck.function_scoped_fixture, HealthCheck.too_slow])
@given(shapes=st.lists(st.one_of(st.tuples(st.integers(1, 20000)), st.tuples(st.integers(1, 90), st.integers(1, 90))),
                       min_size=1, max_size=6),
       pairs=st.lists(st.tuples(st.integers(0, 7), st.integers(0, 7)), min_size=1, max_size=20),
       dts=st.sampled_from([(torch.bfloat16, torch.bfloat16), (torch.float32, torch.float32),
                            (torch.bfloat16, torch.float32), (torch.float32, torch.bfloat16)]),
       speculate=st.booleans(), lineage=st.booleans(), seed=st.integers(0, 2**31 - 1))
def test_population_fuzz(dev, shapes, pairs, dts, speculate, lineage, seed):
    """ops.slerp_population (r5: the needed-sums passes, member-major or co-located, the triangle
    fallback) on random layouts with 1,024-element chunks, random pair graphs over up to 8 members
    (self pairs, repeats, reversals, isolated members), every dtype route, lineage or mixed members
    (both branches), both forms: every child and its dots bit-identical to edt_slerp_merge."""
    from evolutionarydistributedtraining_amd import ops
    from evolutionarydistributedtraining_amd.params import ParamLayout
    in_dt, out_dt = dts
    layout = ParamLayout(shapes)
    n = layout.total
    M = max(max(p) for p in pairs) + 1
    g = torch.Generator().manual_seed(seed)
    base = torch.randn(n, generator=g) * 0.02
    members = [(base + torch.randn(n, generator=g) * 0.02 * (0.005 if lineage or m % 2 else 0.3)).to(in_dt).to(dev)
               for m in range(M)]
    t = torch.rand(len(shapes), generator=g, dtype=torch.float64).to(dev)
    plan = ops.make_slerp_plan(layout.offsets, dev, chunk_elems=1024)
    outs = [torch.full((n,), float("nan"), dtype=out_dt, device=dev) for _ in pairs]
    dots = ops.slerp_population(plan, members, pairs, outs, t, speculate=speculate).clone()
    want = torch.empty(n, dtype=out_dt, device=dev)
    for q, (i, j) in enumerate(pairs):
        ops.slerp_arena(plan, members[i], members[j], want, t, speculate=False)
        torch.cuda.synchronize()
        assert torch.equal(bits(outs[q]), bits(want)), (q, i, j, speculate)
        assert torch.equal(dots[q][:plan.nseg].cpu(), plan.dots[:plan.nseg].cpu()), (q, i, j)
