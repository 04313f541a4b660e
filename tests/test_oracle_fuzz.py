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
