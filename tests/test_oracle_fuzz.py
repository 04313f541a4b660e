"""Pin the oracle's scalar handling against real torch on this host (CPU, hypothesis): the
reference's outer step is torch code (EDT_LM/diloco.py:238-289: a per-tensor running sum of
(trained - base) / K, `p.grad = -sum`, torch.optim.SGD), so running that loop with torch itself
(oracle.torch_loop_outer_step restates it op for op) is ground truth for ANY optimiser scalars,
not only the golden cases' 0.7 / 0.9. The oracle must match it bit for bit: fp32 everywhere, bf16
with torch's scalar-tail model for this host's vector width (tensors below torch's parallel grain,
so the thread count does not enter). The GPU fuzz (test_gpu_fuzz.py) then ties the kernels to the
oracle over the same scalar space."""
import pytest
import torch
from hypothesis import HealthCheck, given, settings
from hypothesis import strategies as st

FUZZ = settings(max_examples=150, deadline=None, derandomize=True,
                suppress_health_check=[HealthCheck.function_scoped_fixture, HealthCheck.too_slow])
VEC = {"AVX512": 32, "AVX2": 16}.get(torch.backends.cpu.get_cpu_capability())


@pytest.mark.skipif(VEC is None, reason="torch CPU capability without a known bf16 vector width")
@FUZZ
@given(numels=st.lists(st.integers(1, 3000), min_size=1, max_size=4), K=st.integers(1, 6),
       dt=st.sampled_from([torch.float32, torch.bfloat16]),
       lr=st.floats(1e-4, 2.0), mu=st.one_of(st.just(0.0), st.floats(0.0, 0.999)), nesterov=st.booleans(),
       gens=st.integers(1, 3), seed=st.integers(0, 2**31 - 1))
def test_oracle_matches_torch_for_any_scalars(oracle, numels, K, dt, lr, mu, nesterov, gens, seed):
    if nesterov and mu == 0:
        nesterov = False
    g = torch.Generator().manual_seed(seed)
    base = [(torch.randn(n, generator=g) * 0.02).to(dt) for n in numels]
    flat = torch.cat(base).clone()
    mom = torch.zeros_like(flat)
    tail = oracle.torch_cpu_tail_mask(numels, vec_elems=VEC) if dt == torch.bfloat16 else None
    opt = None
    for gen in range(gens):
        workers = [[(p.float() + torch.randn(p.shape, generator=g) * 1e-3 * (gen + 1)).to(dt) for p in base]
                   for _ in range(K)]
        opt = oracle.torch_loop_outer_step(base, workers, opt, lr, mu, nesterov)      # torch itself
        oracle.outer_step(flat, [torch.cat(w) for w in workers], mom if mu else None, gen > 0, lr, mu, nesterov,
                          tail)
        got = torch.cat([p.detach().reshape(-1) for p in base])
        bits = (lambda t: t.view(torch.int32)) if dt == torch.float32 else (lambda t: t.view(torch.int16))
        assert torch.equal(bits(got), bits(flat)), gen


def _reference_pair_merge(b1s, b2s, m1s, m2s, parent_mom, lr, mu, nesterov):
    """EDT_LM/train/crossover.py's child, with torch itself: run_linear_merge_5050's
    lerp(0.5) = (1 - t) * v0 + t * v1 per tensor (:50-51, :150-162), then run_sgd (:166-237):
    delta = ((p1 - base) + (p2 - base)) / 2 accumulated into zeros, grad = -delta, SGD with
    parent 1's outer_optim.pt loaded when it exists (the nested-dict merge keeps state1's entries)."""
    base = [((1 - 0.5) * a + 0.5 * b).clone() for a, b in zip(b1s, b2s)]
    acc = [torch.zeros_like(p) for p in base]
    for i, (p, p1, p2) in enumerate(zip(base, m1s, m2s)):
        acc[i] += ((p1 - p) + (p2 - p)) / 2
    for p, a in zip(base, acc):
        p.grad = -a
    opt = torch.optim.SGD(base, lr=lr, momentum=mu, nesterov=nesterov)
    if parent_mom is not None:
        sd = opt.state_dict()
        sd["state"] = {i: {"momentum_buffer": m.clone()} for i, m in enumerate(parent_mom)}
        opt.load_state_dict(sd)
    opt.step()
    mom = [opt.state[p]["momentum_buffer"] for p in base] if mu else None
    return base, mom


@pytest.mark.skipif(VEC is None, reason="torch CPU capability without a known bf16 vector width")
@FUZZ
@given(numels=st.lists(st.integers(1, 3000), min_size=1, max_size=4),
       dt=st.sampled_from([torch.float32, torch.bfloat16]),
       lr=st.floats(1e-4, 2.0), mu=st.one_of(st.just(0.0), st.floats(1e-3, 0.999)), nesterov=st.booleans(),
       has=st.booleans(), seed=st.integers(0, 2**31 - 1))
def test_oracle_pair_merge_matches_torch_for_any_scalars(oracle, numels, dt, lr, mu, nesterov, has, seed):
    if nesterov and mu == 0:
        nesterov = False
    if mu == 0:
        has = False
    g = torch.Generator().manual_seed(seed)
    b1s, b2s = ([(torch.randn(n, generator=g) * 0.02).to(dt) for n in numels] for _ in range(2))
    m1s = [(b.float() + torch.randn(b.shape, generator=g) * 1e-3).to(dt) for b in b1s]
    m2s = [(b.float() + torch.randn(b.shape, generator=g) * 1e-3).to(dt) for b in b2s]
    pm = [(torch.randn(n, generator=g) * 1e-3).to(dt) for n in numels] if has else None
    want, want_m = _reference_pair_merge(b1s, b2s, m1s, m2s, pm, lr, mu, nesterov)
    out = torch.empty(sum(numels), dtype=dt)
    mom = torch.cat(pm).clone() if has else torch.zeros(sum(numels), dtype=dt)
    tail = oracle.torch_cpu_tail_mask(numels, vec_elems=VEC) if dt == torch.bfloat16 else None
    oracle.pair_merge(torch.cat(b1s), torch.cat(b2s), torch.cat(m1s), torch.cat(m2s), out, mom if mu else None,
                      has, lr, mu, nesterov, tail)
    bits = (lambda t: t.view(torch.int32)) if dt == torch.float32 else (lambda t: t.view(torch.int16))
    assert torch.equal(bits(torch.cat([p.detach() for p in want])), bits(out))
    if mu:
        assert torch.equal(bits(torch.cat(want_m)), bits(mom))
