"""HIP kernels vs the CPU oracle and the reference's golden vectors (needs an MI355X).

Bars (stated per test):
  * vs the oracle in its vectorised-torch semantics (tail=None): bit-exact, every element.
  * vs the reference goldens: fp32 regimes bit-exact; bf16 regime bit-exact except on the
    elements torch's CPU kernels send down their scalar tail (oracle.torch_cpu_tail_mask), where
    the reference itself rounds add(..., alpha) twice (the oracle reproduces both forms bit for
    bit, tests/test_oracle_golden.py). There the SGD direction u differs by <= 1 bf16 ulp, so
    |diff| <= 2 ulp(theta_out) + 2 ulp(|theta_out - theta_in|).
  * SLERP: the reference's dot is an fp32 BLAS/pairwise sum; ours is an fp64 sum. Coefficients
    agree to ~1e-6 relative, so |out - ref| <= 2e-6 * (|c0 v0| + |c1 v1|) + 1e-30.
"""
import json
import os

import pytest
import torch

from tests.golden_data import GOLDEN_DIR, bits, flat

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

pytestmark = pytest.mark.gpu

with open(os.path.join(GOLDEN_DIR, "manifest.json")) as _f:
    _M = json.load(_f)


@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    return torch.device("cuda:0")


@pytest.fixture(scope="module")
def ops():
    from evolutionarydistributedtraining_amd import ops as o
    return o


def ulp_bf16(x: torch.Tensor) -> torch.Tensor:
    """Size of one bf16 ulp at |x| (as float32)."""
    a = x.float().abs().clamp_min(torch.finfo(torch.bfloat16).tiny)
    e = torch.floor(torch.log2(a))
    return torch.exp2(e - 7)


def update_tol(want, theta_in):
    """Bound for a result whose SGD direction differs by one bf16 rounding."""
    step = (want.float() - theta_in.float()).abs()
    return 2 * ulp_bf16(want) + 2 * ulp_bf16(step)


def assert_matches_reference(got, want, tail, what, theta_in):
    if got.dtype == torch.float32:
        assert torch.equal(bits(got), bits(want)), f"{what}: fp32 not bit-exact"
        return
    diff = bits(got) != bits(want)
    outside = diff & (tail == 0)
    assert not outside.any(), f"{what}: {int(outside.sum())} mismatches outside torch's scalar tails"
    if diff.any():
        d = (got.float() - want.float()).abs()[diff]
        assert (d <= update_tol(want, theta_in)[diff] * 1.0001).all(), f"{what}: tail diff too large"


@pytest.mark.parametrize("idx", range(len(_M["diloco"])))
def test_diloco_golden(golden, oracle, dev, ops, idx):
    c = golden.diloco_cases()[idx]
    T = len(c["shapes"])
    numels = [int(torch.Size(s).numel()) for s in c["shapes"]]
    tail = oracle.torch_cpu_tail_mask(numels)
    prev_buf = None
    for step in c["steps"]:
        pre = step["prefix"]
        theta = flat(golden.tlist("diloco", f"{pre}/base", T)).contiguous()
        workers = [flat(golden.tlist("diloco", f"{pre}/worker{k}", T)).contiguous() for k in range(c["K"])]
        mu = c["momentum"]
        if mu == 0:
            mom, has = None, False
        elif prev_buf is None:
            mom, has = torch.zeros_like(theta), False
        else:
            mom, has = prev_buf.clone(), True
        th_d = theta.to(dev)
        theta_in = theta.clone()
        mom_d = None if mom is None else mom.to(dev)
        ops.outer_step(th_d, [w.to(dev) for w in workers], mom_d, has, c["lr"], mu, c["nesterov"])
        # oracle, vectorised semantics: bit-exact on every element
        oracle.outer_step(theta, workers, mom, has, c["lr"], mu, c["nesterov"])
        got = th_d.cpu()
        assert torch.equal(bits(got), bits(theta)), f"{pre}: kernel != oracle"
        want = flat(golden.tlist("diloco", f"{pre}/out_theta", T))
        assert_matches_reference(got, want, tail, pre, theta_in)
        if step["has_out_buf"]:
            gb = mom_d.cpu()
            assert torch.equal(bits(gb), bits(mom)), f"{pre}: momentum kernel != oracle"
            assert torch.equal(bits(gb), bits(flat(golden.tlist("diloco", f"{pre}/out_buf", T))))
            prev_buf = gb


@pytest.mark.parametrize("idx", range(len(_M["diloco"])))
def test_diloco_golden_tensor_list(golden, oracle, dev, ops, idx):
    """The tensor-list launch (edt_outer_step_list) on the golden cases: one device tensor per
    parameter, as `list(model.parameters())` hands them over; same bars as the flat launch."""
    c = golden.diloco_cases()[idx]
    T = len(c["shapes"])
    numels = [int(torch.Size(s).numel()) for s in c["shapes"]]
    tail = oracle.torch_cpu_tail_mask(numels)
    prev_buf = None
    for step in c["steps"]:
        pre = step["prefix"]
        base = golden.tlist("diloco", f"{pre}/base", T)
        workers = [golden.tlist("diloco", f"{pre}/worker{k}", T) for k in range(c["K"])]
        mu = c["momentum"]
        theta = flat(base).contiguous()
        theta_in = theta.clone()
        if mu == 0:
            mom, has = None, False
        elif prev_buf is None:
            mom, has = torch.zeros_like(theta), False
        else:
            mom, has = prev_buf.clone(), True
        th_d = [t.contiguous().to(dev) for t in base]
        ws_d = [[t.contiguous().to(dev) for t in w] for w in workers]
        mom_d = None if mom is None else [m.contiguous().to(dev) for m in
                                          torch.split(mom, numels)]
        ops.outer_step_list(th_d, ws_d, mom_d, has, c["lr"], mu, c["nesterov"])
        oracle.outer_step(theta, [flat(w).contiguous() for w in workers], mom, has, c["lr"], mu, c["nesterov"])
        got = flat([t.cpu() for t in th_d])
        assert torch.equal(bits(got), bits(theta)), f"{pre}: list kernel != oracle"
        assert_matches_reference(got, flat(golden.tlist("diloco", f"{pre}/out_theta", T)), tail, pre, theta_in)
        if step["has_out_buf"]:
            gb = flat([m.cpu() for m in mom_d])
            assert torch.equal(bits(gb), bits(mom))
            prev_buf = gb


@pytest.mark.parametrize("gdt,wdt", [(torch.float32, torch.float32), (torch.float32, torch.bfloat16),
                                     (torch.bfloat16, torch.bfloat16)])
@pytest.mark.parametrize("K", [1, 3, 5, 8, 32])
def test_outer_step_list_vs_oracle(oracle, dev, ops, gdt, wdt, K):
    """Ragged tensor lists: empty tensors, sizes around the 32768-element chunk and the 8-element
    vector, a tensor off a 16-byte boundary (scalar body), separate allocations per worker."""
    numels = [0, 1, 7, 8, 9, 32767, 32768, 32769, 100_003, 0, 65536 * 3 + 5, 13]
    n = sum(numels)
    theta, workers, mom = _rand_case(n, K, gdt, wdt, seed=K + 17)
    offs = [0]
    for x in numels:
        offs.append(offs[-1] + x)

    def split(v):   # separate allocations; tensor 4 starts 2 elements into its buffer
        out = []
        for t, (a, b) in enumerate(zip(offs, offs[1:])):
            if t == 4:
                buf = torch.empty(b - a + 2, dtype=v.dtype, device=dev)
                buf[2:].copy_(v[a:b])
                out.append(buf[2:])
            else:
                out.append(v[a:b].to(dev).clone())
        return out

    for has, (lr, mu, nest) in [(False, (0.7, 0.9, True)), (True, (0.7, 0.9, True)),
                                (True, (0.5, 0.8, False)), (False, (1.0, 0.0, False))]:
        th, m = theta.clone(), mom.clone()
        th_d, m_d, ws_d = split(th), split(m), [split(w) for w in workers]
        ops.outer_step_list(th_d, ws_d, m_d if mu else None, has, lr, mu, nest)
        oracle.outer_step(th, workers, m if mu else None, has, lr, mu, nest)
        assert torch.equal(bits(torch.cat([t.cpu() for t in th_d])), bits(th)), (has, lr, mu, nest)
        if mu:
            assert torch.equal(bits(torch.cat([t.cpu() for t in m_d])), bits(m))


def _rand_case(n, K, gdt, wdt, seed):
    g = torch.Generator().manual_seed(seed)
    theta = (torch.randn(n, generator=g) * 0.02).to(gdt)
    workers = [(theta.float() + torch.randn(n, generator=g) * 1e-3).to(wdt) for _ in range(K)]
    mom = (torch.randn(n, generator=g) * 1e-3).to(gdt)
    return theta, workers, mom


REGIMES = [(torch.float32, torch.float32), (torch.float32, torch.bfloat16), (torch.bfloat16, torch.bfloat16)]


# the large size with representative populations only
OUTER_CASES = [(n, K) for n in (1, 7, 8, 9, 4097, 1_000_003) for K in (1, 2, 3, 4, 5, 8, 16, 32, 33, 48, 64, 65, 100, 129)
               if n != 1_000_003 or K in (3, 8, 48, 65)]


@pytest.mark.parametrize("gdt,wdt", REGIMES)
@pytest.mark.parametrize("n,K", OUTER_CASES)
def test_outer_step_vs_oracle(oracle, dev, ops, gdt, wdt, K, n):
    """K > 64 runs as chained launches carrying the running sum (edt_outer_step_ws)."""
    theta, workers, mom = _rand_case(n, K, gdt, wdt, seed=K * 1000 + n)
    for has, (lr, mu, nest) in [(False, (0.7, 0.9, True)), (True, (0.7, 0.9, True)),
                                (True, (0.5, 0.8, False)), (False, (1.0, 0.0, False))]:
        th, m = theta.clone(), mom.clone()
        th_d, m_d = th.to(dev), m.to(dev)
        ops.outer_step(th_d, [w.to(dev) for w in workers], m_d if mu else None, has, lr, mu, nest)
        oracle.outer_step(th, workers, m if mu else None, has, lr, mu, nest)
        assert torch.equal(bits(th_d.cpu()), bits(th)), (has, lr, mu, nest)
        if mu:
            assert torch.equal(bits(m_d.cpu()), bits(m))


@pytest.mark.parametrize("gdt,wdt", REGIMES)
def test_outer_step_misaligned_views(oracle, dev, ops, gdt, wdt):
    """Views starting off a 16-byte boundary take the scalar path; results are unchanged."""
    n, K = 3001, 3
    theta, workers, mom = _rand_case(n + 1, K, gdt, wdt, seed=7)
    th_d = theta.to(dev)[1:]
    ws_d = [w.to(dev)[1:] for w in workers]
    m_d = mom.to(dev)[1:]
    ops.outer_step(th_d, ws_d, m_d, True, 0.7, 0.9, True)
    th, m = theta[1:].clone(), mom[1:].clone()
    oracle.outer_step(th, [w[1:].clone() for w in workers], m, True, 0.7, 0.9, True)
    assert torch.equal(bits(th_d.cpu()), bits(th))
    assert torch.equal(bits(m_d.cpu()), bits(m))


def test_outer_step_edge_values(oracle, dev, ops):
    """Signed zeros, identical replicas, subnormals, large values and deltas."""
    vals = torch.tensor([0.0, -0.0, 1e-40, -1e-40, 3.0, -2.5, 1e30, -3e38, 1.0, 0.02])
    theta = vals.clone()
    workers = [vals.clone(), vals + torch.tensor([1e-3, -0.0, 1e-40, 0, 0.25, 0, 1e29, 0, -1e-7, 5e-4])]
    for gdt in (torch.float32, torch.bfloat16):
        th, ws = theta.to(gdt), [w.to(gdt) for w in workers]
        m = torch.zeros_like(th)
        th_d, m_d = th.to(dev), m.to(dev)
        ops.outer_step(th_d, [w.to(dev) for w in ws], m_d, False, 0.7, 0.9, True)
        oracle.outer_step(th, ws, m, False, 0.7, 0.9, True)
        assert torch.equal(bits(th_d.cpu()), bits(th))


@pytest.mark.parametrize("gdt,wdt", REGIMES)
def test_partial_then_sgd(oracle, dev, ops, gdt, wdt):
    """Sharded form: fp32 partial sums + sgd_apply == fused step (fp32 regimes: bit-exact,
    the fp32 partial accumulates in the same order; bf16: the fused form rounds the running sum
    to bf16 after every worker, as the reference does, so the SGD direction differs by a few
    bf16 ulps of its terms: |diff| <= 2 ulp(theta_out) + 4 ulp(|update| + lr (|buf'| + mu |buf|)))."""
    n, K = 100_003, 4
    theta, workers, mom = _rand_case(n, K, gdt, wdt, seed=11)
    th_d, m_d = theta.to(dev), mom.to(dev)
    ws_d = [w.to(dev) for w in workers]
    acc = torch.empty(n, dtype=torch.float32, device=dev)
    ops.delta_partial(th_d, ws_d[:2], K, acc, accumulate=False)
    ops.delta_partial(th_d, ws_d[2:], K, acc, accumulate=True)
    ops.sgd_apply(th_d, acc, m_d, True, 0.7, 0.9, True)
    th, m = theta.clone(), mom.clone()
    oracle.outer_step(th, workers, m, True, 0.7, 0.9, True)
    got = th_d.cpu()
    if gdt == torch.float32:
        assert torch.equal(bits(got), bits(th))
    else:   # fp32 running sum vs the reference's bf16-rounded one: the direction differs slightly
        d = (got.float() - th.float()).abs()
        scale = (th.float() - theta.float()).abs() + 0.7 * (m.float().abs() + 0.9 * mom.float().abs())
        assert (d <= (2 * ulp_bf16(th) + 4 * ulp_bf16(scale)) * 1.0001).all()


@pytest.mark.parametrize("idx", range(len(_M["pair_merge"])))
def test_pair_merge_golden(golden, oracle, dev, ops, idx):
    from tests.test_oracle_golden import pair_inputs
    c = golden.pair_cases()[idx]
    p = pair_inputs(golden, c)
    tail = oracle.torch_cpu_tail_mask([int(torch.Size(s).numel()) for s in c["shapes"]])
    n = p["b1"].numel()
    out_d = torch.empty(n, dtype=p["bdt"], device=dev)
    mom_d = None if p["mom"] is None else p["mom"].to(dev)
    ops.pair_merge(p["b1"].to(dev), p["b2"].to(dev), p["m1"].to(dev), p["m2"].to(dev), out_d, mom_d,
                   p["has"], p["lr"], p["mu"], p["nesterov"])
    out = torch.empty(n, dtype=p["bdt"])
    mom = None if p["mom"] is None else p["mom"].clone()
    oracle.pair_merge(p["b1"], p["b2"], p["m1"], p["m2"], out, mom, p["has"], p["lr"], p["mu"], p["nesterov"])
    assert torch.equal(bits(out_d.cpu()), bits(out)), "kernel != oracle"
    assert_matches_reference(out_d.cpu(), p["want_theta"], tail, c["name"], p["want_base"])
    if p["want_buf"] is not None:
        assert torch.equal(bits(mom_d.cpu()), bits(p["want_buf"].to(p["bdt"])))
    # merged base alone (run_linear_merge_5050)
    base_d = ops.lerp(0.5, p["b1"].to(dev), p["b2"].to(dev)).to(p["bdt"])
    assert torch.equal(bits(base_d.cpu()), bits(p["want_base"]))
    # base-given form (run_sgd on a merged base model)
    out2 = torch.empty_like(out_d)
    mom2 = None if p["mom"] is None else pair_inputs(golden, c)["mom"].to(dev)
    ops.pair_merge(base_d, None, p["m1"].to(dev), p["m2"].to(dev), out2, mom2, p["has"], p["lr"], p["mu"],
                   p["nesterov"])
    assert torch.equal(bits(out2.cpu()), bits(out))
    # donor form (edt_pair_merge_to): carried momentum read from a separate buffer, left intact
    if p["mom"] is not None:
        donor = pair_inputs(golden, c)["mom"].to(dev)
        keep = donor.clone()
        out3 = torch.empty_like(out_d)
        mom3 = torch.full_like(donor, float("nan"))
        ops.pair_merge(p["b1"].to(dev), p["b2"].to(dev), p["m1"].to(dev), p["m2"].to(dev), out3, mom3,
                       p["has"], p["lr"], p["mu"], p["nesterov"], momentum_in=donor)
        assert torch.equal(bits(out3.cpu()), bits(out))
        assert torch.equal(bits(mom3.cpu()), bits(mom_d.cpu()))
        assert torch.equal(bits(donor.cpu()), bits(keep.cpu()))


@pytest.mark.parametrize("in_dt,cdt,out_dt", [(torch.float32, torch.float32, torch.float32),
                                              (torch.bfloat16, torch.bfloat16, torch.bfloat16),
                                              (torch.bfloat16, torch.float32, torch.float32),
                                              (torch.bfloat16, torch.float32, torch.bfloat16)])
@pytest.mark.parametrize("t", [0.0, 0.5, 0.43333333333333335, 1.0])
def test_lerp_vs_oracle(oracle, dev, ops, in_dt, cdt, out_dt, t):
    g = torch.Generator().manual_seed(3)
    n = 70_001
    v0 = (torch.randn(n, generator=g) * 0.02).to(in_dt)
    v1 = (torch.randn(n, generator=g) * 0.02).to(in_dt)
    out_d = torch.empty(n, dtype=out_dt, device=dev)
    ops.lerp(t, v0.to(dev), v1.to(dev), out=out_d, compute_dtype=cdt)
    want = oracle.lerp(t, v0, v1, compute_dtype=cdt, out_dtype=out_dt)
    assert torch.equal(bits(out_d.cpu()), bits(want))


def _slerp_tol(c0, c1, v0, v1):
    return 2e-6 * (abs(float(c0)) * v0.float().abs() + abs(float(c1)) * v1.float().abs()) + 1e-30


def test_slerp_golden(golden, oracle, dev, ops):
    """Each golden SLERP case as a one-segment arena: branch, dot and output vs the reference."""
    t = golden.tensors("slerp")
    for c in golden.slerp_cases():
        v0, v1 = t[f"{c['inputs']}/v0"].reshape(-1), t[f"{c['inputs']}/v1"].reshape(-1)
        want = t[f"{c['name']}/out"].reshape(-1)
        n = v0.numel()
        plan = ops.make_slerp_plan([0, n], dev, chunk_elems=1024)
        out_d = torch.empty(n, dtype=torch.float32, device=dev)
        ops.slerp_arena(plan, v0.to(dev), v1.to(dev), out_d,
                        torch.tensor([c["t"]], dtype=torch.float64, device=dev))
        dot = plan.dots[0].item()
        assert abs(dot - c["ref_dot"]) <= 2e-6, (c["name"], dot, c["ref_dot"])
        assert (abs(dot) > 0.9995) == c["lerp_branch"], c["name"]
        c0, c1, _ = oracle.slerp_coefficients(c["t"], v0, v1)
        got = out_d.cpu()
        err = (got - want).abs()
        assert (err <= _slerp_tol(c0, c1, v0, v1)).all(), (c["name"], err.max().item())
        if c["lerp_branch"]:
            assert torch.equal(bits(got), bits(want)), c["name"]   # same coefficients -> exact


@pytest.mark.parametrize("in_dt,out_dt", [(torch.float32, torch.float32), (torch.bfloat16, torch.float32),
                                          (torch.bfloat16, torch.bfloat16)])
def test_slerp_multi_segment(oracle, dev, ops, in_dt, out_dt):
    """Ragged multi-tensor arena (empty, 1-element, odd, chunk-crossing segments), per-segment t."""
    g = torch.Generator().manual_seed(5)
    sizes = [0, 1, 7, 33, 4096, 70_001, 0, 129, 200_000]
    offs = [0]
    for s in sizes:
        offs.append(offs[-1] + s)
    v0 = torch.randn(offs[-1], generator=g) * 0.02
    v1 = v0 + torch.randn(offs[-1], generator=g) * 0.02 * 0.05
    v1[offs[4]:offs[5]] = 2 * v0[offs[4]:offs[5]]               # parallel -> lerp branch
    v0[offs[7]:offs[8]] = 0                                      # zero tensor
    v0, v1 = v0.to(in_dt), v1.to(in_dt)
    ts = torch.tensor([0.5, 0.0, 1.0, 0.43333333333333335, 0.5, 0.7, 0.5, 0.2, 0.9], dtype=torch.float64)
    plan = ops.make_slerp_plan(offs, dev, chunk_elems=4096)
    out_d = torch.empty(offs[-1], dtype=out_dt, device=dev)
    ops.slerp_arena(plan, v0.to(dev), v1.to(dev), out_d, ts.to(dev))
    got = out_d.cpu().float()
    coef = plan.coef.cpu()
    for s in range(len(sizes)):
        a, b = offs[s], offs[s + 1]
        if a == b:
            continue
        want = oracle.slerp(float(ts[s]), v0[a:b], v1[a:b])
        rc0, rc1, rdot = oracle.slerp_coefficients(float(ts[s]), v0[a:b], v1[a:b])
        assert abs(float(rdot) - plan.dots[s].item()) < 1e-5, s
        c0, c1 = coef[s].tolist()
        # our result is the fp32 blend with our coefficients; the reference's with its own
        tol = 1.01 * (abs(c0 - float(rc0)) * v0[a:b].float().abs() + abs(c1 - float(rc1)) * v1[a:b].float().abs())
        tol = tol + _slerp_tol(c0, c1, v0[a:b], v1[a:b])
        if out_dt == torch.bfloat16:
            want = want.bfloat16().float()
            tol = tol + ulp_bf16(want)
        assert ((got[a:b] - want).abs() <= tol).all(), s


@pytest.mark.parametrize("in_dt,out_dt", [(torch.float32, torch.float32), (torch.bfloat16, torch.float32),
                                          (torch.bfloat16, torch.bfloat16)])
def test_slerp_list_matches_arena(dev, ops, in_dt, out_dt):
    """The tensor-list SLERP (separate tensors, relative chunk starts) is bit-identical to the
    arena SLERP on the same data: same chunking, same fixed-order sums. Also in place into v0."""
    from evolutionarydistributedtraining_amd.merge import slerp_tensors
    g = torch.Generator().manual_seed(11)
    sizes = [0, 1, 7, 33, 4096, 70_001, 0, 129, 200_000]
    offs = [0]
    for x in sizes:
        offs.append(offs[-1] + x)
    v0 = (torch.randn(offs[-1], generator=g) * 0.02).to(in_dt)
    v1 = (v0.float() + torch.randn(offs[-1], generator=g) * 1e-3).to(in_dt)
    ts = torch.tensor([0.5, 0.0, 1.0, 0.3, 0.5, 0.7, 0.5, 0.2, 0.9], dtype=torch.float64)
    plan = ops.make_slerp_plan(offs, dev)              # default chunking, as slerp_tensors uses
    ref = torch.empty(offs[-1], dtype=out_dt, device=dev)
    ops.slerp_arena(plan, v0.to(dev), v1.to(dev), ref, ts.to(dev))
    ref_dots = plan.dots.cpu().clone()
    a0 = [v0[a:b].to(dev).clone() for a, b in zip(offs, offs[1:])]
    a1 = [v1[a:b].to(dev).clone() for a, b in zip(offs, offs[1:])]
    outs = [torch.empty(x, dtype=out_dt, device=dev) for x in sizes]
    lplan = ops.make_slerp_plan(offs, dev, relative=True)
    ops.slerp_list(lplan, a0, a1, outs, ts.to(dev))
    assert torch.equal(bits(torch.cat([o.cpu() for o in outs])), bits(ref.cpu()))
    assert torch.equal(lplan.dots.cpu(), ref_dots)
    if in_dt == out_dt:                     # merged into the first parent's own tensors
        res = slerp_tensors(list(zip(a0, a1)), ts.tolist(), out=a0)
        assert res is a0 or all(r.data_ptr() == x.data_ptr() for r, x in zip(res, a0))
        assert torch.equal(bits(torch.cat([x.cpu() for x in a0])), bits(ref.cpu()))


@pytest.mark.parametrize("in_dt,out_dt", [(torch.float32, torch.float32), (torch.bfloat16, torch.float32),
                                          (torch.bfloat16, torch.bfloat16)])
def test_slerp_list_speculative_matches_two_pass(dev, ops, in_dt, out_dt):
    """edt_slerp_merge_list_speculative (lerp-branch outputs written in the sums pass over the
    tensors where they lie, SLERP-branch tensors blended again) is bit-identical to the two-pass
    list form and to the arena form: outputs and dots, tensors on both sides of the threshold,
    ragged and empty tensors, a zero tensor; the adaptive choice follows the previous dots; an
    output equal to its parent is refused by the entry and handled by the two-pass form."""
    from evolutionarydistributedtraining_amd import _lib as L
    g = torch.Generator().manual_seed(79)
    sizes = [0, 1, 7, 33, 4096, 70_001, 0, 129, 200_003, 65_536, 131_073]
    rel = [0.1, 0.001, 0.2, 0.001, 0.05, 0.005, 0.1, 0.3, 0.002, 0.02, 0.0005]
    offs = [0]
    for x in sizes:
        offs.append(offs[-1] + x)
    v0 = torch.randn(offs[-1], generator=g) * 0.02
    v1 = v0.clone()
    for s_, r in enumerate(rel):
        a, b = offs[s_], offs[s_ + 1]
        v1[a:b] += torch.randn(b - a, generator=g) * 0.02 * r
    v0[offs[7]:offs[8]] = 0
    ts = torch.tensor([0.5, 0.0, 1.0, 0.43, 0.5, 0.7, 0.5, 0.2, 0.9, 0.3, 0.6], dtype=torch.float64).to(dev)
    plan = ops.make_slerp_plan(offs, dev)
    ref = torch.empty(offs[-1], dtype=out_dt, device=dev)
    ops.slerp_arena(plan, v0.to(in_dt).to(dev), v1.to(in_dt).to(dev), ref, ts, speculate=False)
    ref_dots = plan.dots.cpu().clone()
    d = ref_dots[:len(sizes)].abs()
    assert (d > 0.9995).any() and (d <= 0.9995).any()
    a0 = [v0[a:b].to(in_dt).to(dev).clone() for a, b in zip(offs, offs[1:])]
    a1 = [v1[a:b].to(in_dt).to(dev).clone() for a, b in zip(offs, offs[1:])]
    lplan = ops.make_slerp_plan(offs, dev, relative=True)
    for speculate in (False, True, None):
        outs = [torch.full((x,), float("nan"), dtype=out_dt, device=dev) for x in sizes]
        lplan.dots.fill_(float("nan"))
        ops.slerp_list(lplan, a0, a1, outs, ts, speculate=speculate)
        assert torch.equal(bits(torch.cat([o.cpu() for o in outs])), bits(ref.cpu())), speculate
        assert torch.equal(lplan.dots.cpu(), ref_dots), speculate
    if in_dt == out_dt:                     # in place over parent 0: the two-pass list form
        c0 = [x.clone() for x in a0]
        ops.slerp_list(lplan, c0, a1, c0, ts, speculate=True)
        assert torch.equal(bits(torch.cat([x.cpu() for x in c0])), bits(ref.cpu()))
        ws = torch.empty(3 * len(sizes), dtype=torch.int64, device=dev)
        numel = (L.ctypes.c_uint64 * len(sizes))(*sizes)
        redo = torch.empty(len(sizes), dtype=torch.int32, device=dev)
        rc = L.lib().edt_slerp_merge_list_speculative(
            L.ptr_array(a0), L.ptr_array(a1), L.dtype_code(in_dt), L.ptr_array(a0), L.dtype_code(out_dt), numel,
            L.ptr(lplan.chunks), lplan.nchunks, L.ptr(lplan.seg_first), lplan.nseg, L.ptr(ts), 0.9995, 1e-8,
            L.ptr(lplan.partial), L.ptr(lplan.coef), None, L.ptr(redo), L.ptr(ws), ws.numel() * 8,
            L.stream_ptr(dev))
        assert rc != 0 and b"apart" in L.lib().edt_last_error()
        # ... and so is an output that overlaps ANOTHER tensor's parent (tied storage,
        # partial overlap): tensor 3's output inside tensor 4's parent
        outs_x = [torch.empty(x, dtype=out_dt, device=dev) for x in sizes]
        big = a1[4]
        outs_x[3] = big[:sizes[3]] if sizes[3] <= sizes[4] else outs_x[3]
        if sizes[3] <= sizes[4] and in_dt == out_dt:
            rc = L.lib().edt_slerp_merge_list_speculative(
                L.ptr_array(a0), L.ptr_array(a1), L.dtype_code(in_dt), L.ptr_array(outs_x), L.dtype_code(out_dt),
                numel, L.ptr(lplan.chunks), lplan.nchunks, L.ptr(lplan.seg_first), lplan.nseg, L.ptr(ts), 0.9995,
                1e-8, L.ptr(lplan.partial), L.ptr(lplan.coef), None, L.ptr(redo), L.ptr(ws), ws.numel() * 8,
                L.stream_ptr(dev))
            assert rc != 0 and b"overlaps a parent" in L.lib().edt_last_error()
            # refused for the two-pass form as well (its blend would race): edt_slerp_seg_table's
            # in-place rule (r5, in C) — an output may only be exactly its own parent
            with pytest.raises(L.EdtError, match="overlaps another tensor's parent or output"):
                ops.slerp_list(lplan, a0, a1, outs_x, ts)


@pytest.mark.parametrize("in_dt,out_dt", [(torch.float32, torch.float32), (torch.bfloat16, torch.bfloat16)])
@pytest.mark.parametrize("nmem", [1, 2, 3, 5, 8, 11])    # 11: > 8 distinct parents (speculative only)
def test_slerp_population_matches_per_child(dev, ops, in_dt, out_dt, nmem):
    """edt_slerp_population (one Gram pass over the members, then per-child coefficients and
    blends) is bit-identical to edt_slerp_merge per child: same sums, coefficients and outputs.
    Ragged segments, a zero segment, a parallel pair (lerp branch), self-pairs."""
    g = torch.Generator().manual_seed(40 + nmem)
    sizes = [0, 1, 7, 33, 4096, 70_001, 0, 129, 200_003]
    offs = [0]
    for x in sizes:
        offs.append(offs[-1] + x)
    base = torch.randn(offs[-1], generator=g) * 0.02
    # members 0-2 near each other (lerp branch on most segments), the rest farther (SLERP branch)
    mem = [base + torch.randn(offs[-1], generator=g) * (1e-5 if m < 3 else 1e-3) * (m + 1) for m in range(nmem)]
    if nmem > 1:
        mem[1][offs[4]:offs[5]] = 2 * mem[0][offs[4]:offs[5]]      # parallel -> lerp branch
    mem[0][offs[7]:offs[8]] = 0                                      # zero tensor
    mem = [m.to(in_dt).to(dev) for m in mem]
    pairs = [(i % nmem, (3 * i + 1) % nmem) for i in range(max(nmem, 3))] + [(0, 0)]
    ts = torch.tensor([0.5, 0.0, 1.0, 0.43333333333333335, 0.5, 0.7, 0.5, 0.2, 0.9], dtype=torch.float64).to(dev)
    plan = ops.make_slerp_plan(offs, dev, chunk_elems=4096)
    # speculative: member-major first pass when the distinct parents are <= 8, co-located
    # per-child pass above that
    for spec in ((False, True) if nmem <= 8 else (True,)):
        outs = [torch.full((offs[-1],), float("nan"), dtype=out_dt, device=dev) for _ in pairs]
        dots = ops.slerp_population(plan, mem, pairs, outs, ts, speculate=spec).clone()
        for q, (i, j) in enumerate(pairs):
            want = torch.empty(offs[-1], dtype=out_dt, device=dev)
            ops.slerp_arena(plan, mem[i], mem[j], want, ts, speculate=False)
            assert torch.equal(bits(outs[q].cpu()), bits(want.cpu())), (spec, q, i, j)
            assert torch.equal(dots[q].cpu(), plan.dots[:len(sizes)].cpu()), (spec, q, i, j)


def _pair_graphs():
    import random
    rnd = random.Random(5)
    cases = {
        "ring8": [(c, (c + 1) % 8) for c in range(8)],                       # the bench's ring
        "matching8": [((3 * c + 1) % 8, (5 * c + 2) % 8) for c in range(8)],  # the probe's pairs
        "ring5_selfpair": [(c, (c + 1) % 5) for c in range(5)] + [(2, 2)],
        "path6": [(0, 1), (1, 2), (2, 3), (3, 4), (4, 5), (5, 4)],
        "two_cycles": [(0, 1), (1, 2), (2, 0), (3, 4), (4, 5), (5, 6), (6, 3)],
        "star": [(0, 1), (0, 2), (0, 3), (3, 0), (4, 5)],
        "cycle_plus_pair": [(0, 1), (1, 2), (2, 3), (3, 0), (4, 5), (5, 5), (6, 6)],
        "triangle": [(0, 1), (1, 2), (2, 0)],
        "ring8_flipped": [(1, 0), (1, 2), (3, 2), (3, 4), (4, 5), (6, 5), (6, 7), (0, 7)],
        "path4": [(0, 1), (2, 1), (2, 3)],
        "ring6_relabelled": [(4, 1), (1, 5), (5, 0), (0, 3), (3, 2), (2, 4)],
        "matching_selfpair": [(0, 1), (1, 0), (2, 3), (3, 2), (4, 4)],
        "path_and_pair": [(0, 1), (1, 2), (3, 4), (4, 3)],
        "single_pair": [(1, 0)],
        "members_unused": [(5, 2), (2, 7), (7, 5)],
    }
    for k in range(6):
        n = rnd.randint(3, 8)
        cases[f"random{k}"] = [(rnd.randrange(n), rnd.randrange(n)) for _ in range(rnd.randint(1, 10))]
    return cases


@pytest.mark.parametrize("speculate", [False, True])
@pytest.mark.parametrize("graph", sorted(_pair_graphs()))
def test_slerp_population_pair_graphs(dev, ops, graph, speculate):
    """edt_slerp_population's stats pass per component of the children's pair graph (r4 ring
    layout; r5: the needed sums — norms, ring dots, up to 4 chords — r6: past the chord slots the
    same pass in the triangle layout); the speculative form takes the member-major pass when every
    component fits its slots, else the co-located pass; every child's
    outputs and dots stay bit-identical to edt_slerp_merge — rings, matchings, paths, several
    cycles, a star, self-pairs, repeated pairs, members no child uses, random graphs, segments on
    both sides of the threshold (the redo blend)."""
    pairs = _pair_graphs()[graph]
    nmem = max(max(p) for p in pairs) + 1
    g = torch.Generator().manual_seed(len(graph) * 7 + nmem)
    sizes = [0, 1, 7, 33, 4096, 70_001, 0, 129, 200_003]
    offs = [0]
    for x in sizes:
        offs.append(offs[-1] + x)
    base = torch.randn(offs[-1], generator=g) * 0.02
    mem = [(base + torch.randn(offs[-1], generator=g) * (1e-5 if m % 2 else 1e-3)).to(torch.bfloat16).to(dev)
           for m in range(nmem)]
    ts = torch.tensor([0.5, 0.0, 1.0, 0.43333333333333335, 0.5, 0.7, 0.5, 0.2, 0.9], dtype=torch.float64).to(dev)
    plan = ops.make_slerp_plan(offs, dev, chunk_elems=4096)
    outs = [torch.full((offs[-1],), float("nan"), dtype=torch.bfloat16, device=dev) for _ in pairs]
    dots = ops.slerp_population(plan, mem, pairs, outs, ts, speculate=speculate).clone()
    for q, (i, j) in enumerate(pairs):
        want = torch.empty(offs[-1], dtype=torch.bfloat16, device=dev)
        ops.slerp_arena(plan, mem[i], mem[j], want, ts, speculate=False)
        assert torch.equal(bits(outs[q].cpu()), bits(want.cpu())), (graph, q, i, j)
        assert torch.equal(dots[q].cpu(), plan.dots[:len(sizes)].cpu()), (graph, q, i, j)


@pytest.mark.parametrize("in_dt,out_dt", [(torch.float32, torch.float32), (torch.bfloat16, torch.float32),
                                          (torch.float32, torch.bfloat16)])
@pytest.mark.parametrize("graph", ["ring8_flipped", "matching_selfpair", "two_cycles"])
def test_slerp_population_pair_graphs_dtypes(dev, ops, graph, in_dt, out_dt):
    """The per-component ring passes (both forms) in the other dtype routes: fp32 members, fp32
    children — every child bit-identical to edt_slerp_merge."""
    pairs = _pair_graphs()[graph]
    nmem = max(max(p) for p in pairs) + 1
    g = torch.Generator().manual_seed(nmem * 11)
    sizes = [1, 7, 33, 4096, 70_001, 129, 20_003]
    offs = [0]
    for x in sizes:
        offs.append(offs[-1] + x)
    base = torch.randn(offs[-1], generator=g) * 0.02
    mem = [(base + torch.randn(offs[-1], generator=g) * (1e-5 if m % 2 else 1e-3)).to(in_dt).to(dev)
           for m in range(nmem)]
    ts = torch.tensor([0.0, 1.0, 0.43333333333333335, 0.5, 0.7, 0.2, 0.9], dtype=torch.float64).to(dev)
    plan = ops.make_slerp_plan(offs, dev, chunk_elems=4096)
    for speculate in (False, True):
        outs = [torch.full((offs[-1],), float("nan"), dtype=out_dt, device=dev) for _ in pairs]
        dots = ops.slerp_population(plan, mem, pairs, outs, ts, speculate=speculate).clone()
        for q, (i, j) in enumerate(pairs):
            want = torch.empty(offs[-1], dtype=out_dt, device=dev)
            ops.slerp_arena(plan, mem[i], mem[j], want, ts, speculate=False)
            assert torch.equal(bits(outs[q].cpu()), bits(want.cpu())), (graph, speculate, q)
            assert torch.equal(dots[q].cpu(), plan.dots[:len(sizes)].cpu()), (graph, speculate, q)


@pytest.mark.parametrize("threads,vec", [(1, 32), (8, 32), (3, 16)])
def test_list_step_with_tails_equals_flat_tail_step(dev, ops, threads, vec):
    """edt_outer_step_list_tail (r5: the tensor-list step with per-tensor tail masks) equals
    edt_outer_step_tail over the same values packed flat, bit for bit, two generations — tensors
    of ragged sizes, one 4-byte-shifted (the scalar body), all-bf16 Nesterov."""
    from evolutionarydistributedtraining_amd.torchcompat import torch_cpu_tail_bits, torch_cpu_tail_bits_per_tensor
    g = torch.Generator().manual_seed(threads * 100 + vec)
    numels = [70_001, 5, 31, 257 * 160, 33, 300_007, 1]
    bf = torch.bfloat16
    K = 3
    thetas = [(torch.randn(n, generator=g) * 0.02).to(bf).to(dev) for n in numels]
    buf = (torch.randn(numels[2] + 2, generator=g) * 0.02).to(bf).to(dev)
    thetas[2] = buf[2:]                                     # off a 16-byte boundary: the scalar body
    thetas[2].copy_((torch.randn(numels[2], generator=g) * 0.02).to(bf).to(dev))
    workers = [[(t.float() + torch.randn(t.numel(), generator=g).to(dev) * 1e-3).to(bf) for t in thetas]
               for _ in range(K)]
    flat_theta = torch.cat([t.clone() for t in thetas])
    flat_workers = [torch.cat(w) for w in workers]
    moms = [torch.zeros(n, dtype=bf, device=dev) for n in numels]
    flat_mom = torch.zeros(sum(numels), dtype=bf, device=dev)
    tails = torch_cpu_tail_bits_per_tensor(numels, vec_elems=vec, num_threads=threads, device=dev)
    flat_bits = torch_cpu_tail_bits(numels, vec_elems=vec, num_threads=threads, device=dev)
    for gen in range(2):
        ops.outer_step_list(thetas, workers, moms, gen > 0, 0.7, 0.9, True, tails=tails)
        ops.outer_step(flat_theta, flat_workers, flat_mom, gen > 0, 0.7, 0.9, True, tail_bits=flat_bits)
        assert torch.equal(bits(torch.cat(thetas).cpu()), bits(flat_theta.cpu())), gen
        assert torch.equal(bits(torch.cat(moms).cpu()), bits(flat_mom.cpu())), gen


@pytest.mark.parametrize("gdt,wdt", REGIMES)
@pytest.mark.parametrize("n", [1, 8191, 70_001, 1_000_003])
def test_pair_merge_population_matches_per_child(dev, ops, gdt, wdt, n):
    """edt_pair_merge_population (every child in one launch, same-XCD workgroups per chunk) is
    bit-identical to edt_pair_merge_to per child: shared parents, self-pairs, children with and
    without a carried momentum; also through the unaligned (scalar) body."""
    g = torch.Generator().manual_seed(n % 997)
    M = 5
    base = [(torch.randn(n + 1, generator=g) * 0.02).to(wdt).to(dev) for _ in range(M)]
    trained = [(b.float() + torch.randn(n + 1, generator=g).to(dev) * 1e-3).to(wdt) for b in base]
    moms = [(torch.randn(n + 1, generator=g) * 1e-3).to(gdt).to(dev) for _ in range(M)]
    pairs = [(0, 1), (1, 0), (2, 2), (3, 1), (4, 0), (0, 3), (2, 4), (1, 1)]
    for off in (0, 1):                              # off = 1: 4-byte-shifted views -> scalar body
        sl = lambda t: t[off:off + n]
        children, want = [], []
        for c, (i, j) in enumerate(pairs):
            has = c % 3 != 0
            ch = {"b1": sl(base[i]), "b2": sl(base[j]), "m1": sl(trained[i]), "m2": sl(trained[j]),
                  "out": torch.full((n,), float("nan"), dtype=gdt, device=dev),
                  "momentum": torch.full((n,), float("nan"), dtype=gdt, device=dev),
                  "momentum_in": sl(moms[i]) if has else None, "has_momentum": has}
            children.append(ch)
            out = torch.empty(n, dtype=gdt, device=dev)
            mom = torch.empty(n, dtype=gdt, device=dev)
            ops.pair_merge(ch["b1"], ch["b2"], ch["m1"], ch["m2"], out, mom, has, 0.7, 0.9, True,
                           momentum_in=ch["momentum_in"])
            want.append((out, mom))
        ops.pair_merge_population(children, 0.7, 0.9, True)
        for c, (ch, (out, mom)) in enumerate(zip(children, want)):
            assert torch.equal(bits(ch["out"].cpu()), bits(out.cpu())), (off, c)
            assert torch.equal(bits(ch["momentum"].cpu()), bits(mom.cpu())), (off, c)
    for m in moms:                                  # donors are read, never written
        assert not torch.isnan(m.float()).any()


@pytest.mark.parametrize("in_dt,out_dt", [(torch.float32, torch.float32), (torch.bfloat16, torch.float32),
                                          (torch.bfloat16, torch.bfloat16)])
def test_slerp_speculative_matches_two_pass(dev, ops, in_dt, out_dt):
    """edt_slerp_merge_speculative (lerp output written in the stats pass, SLERP-branch segments
    blended again) is bit-identical to edt_slerp_merge: outputs and dots, with segments on both
    sides of the 0.9995 threshold, ragged sizes, a zero segment; the adaptive choice picks the
    cheaper form from the previous merge's dots; an output overlapping a parent is refused by
    the speculative entry and handled by the two-pass form."""
    g = torch.Generator().manual_seed(77)
    sizes = [0, 1, 7, 33, 4096, 70_001, 0, 129, 200_003, 65_536, 131_073]
    offs = [0]
    for x in sizes:
        offs.append(offs[-1] + x)
    v0 = torch.randn(offs[-1], generator=g) * 0.02
    v1 = v0.clone()
    rel = [0.1, 0.001, 0.2, 0.001, 0.05, 0.005, 0.1, 0.3, 0.002, 0.02, 0.0005]   # per segment: far or near
    for s_, r in enumerate(rel):
        a, b = offs[s_], offs[s_ + 1]
        v1[a:b] += torch.randn(b - a, generator=g) * 0.02 * r
    v0[offs[7]:offs[8]] = 0
    v0, v1 = v0.to(in_dt).to(dev), v1.to(in_dt).to(dev)
    ts = torch.tensor([0.5, 0.0, 1.0, 0.43, 0.5, 0.7, 0.5, 0.2, 0.9, 0.3, 0.6], dtype=torch.float64).to(dev)
    plan = ops.make_slerp_plan(offs, dev, chunk_elems=4096)
    ref = torch.empty(offs[-1], dtype=out_dt, device=dev)
    ops.slerp_arena(plan, v0, v1, ref, ts, speculate=False)
    ref_dots = plan.dots.cpu().clone()
    d = ref_dots[:len(sizes)].abs()
    assert (d > 0.9995).any() and (d <= 0.9995).any()          # both branches present
    got = torch.full_like(ref, float("nan"))
    ops.slerp_arena(plan, v0, v1, got, ts, speculate=True)
    assert torch.equal(bits(got.cpu()), bits(ref.cpu()))
    assert torch.equal(plan.dots.cpu(), ref_dots)
    # adaptive: here most elements sit in SLERP-branch segments -> the two-pass form pays
    from evolutionarydistributedtraining_amd.ops import _speculation_pays
    big_slerp = sum(x for x, r in zip(sizes, rel) if r >= 0.02) > 0.67 * offs[-1]
    assert _speculation_pays(plan, v0.element_size(), ref.element_size()) == (not big_slerp)
    if in_dt == out_dt:                                        # in place into parent 1: two-pass form
        v0c = v0.clone()
        ops.slerp_arena(plan, v0c, v1, v0c, ts, speculate=True)
        assert torch.equal(bits(v0c.cpu()), bits(ref.cpu()))
        from evolutionarydistributedtraining_amd import EdtError
        from evolutionarydistributedtraining_amd import _lib as L
        rc = L.lib().edt_slerp_merge_speculative(L.ptr(v0), L.ptr(v1), L.dtype_code(v0), L.ptr(v0), L.dtype_code(v0),
                                                 L.ptr(plan.chunks), plan.nchunks, L.ptr(plan.seg_first), plan.nseg,
                                                 L.ptr(ts), 0.9995, 1e-8, L.ptr(plan.partial), L.ptr(plan.coef), None,
                                                 L.ptr(plan.ws("redo", plan.nseg, torch.int32)), v0.numel(),
                                                 L.stream_ptr(dev))
        assert rc != 0
        with pytest.raises(EdtError):
            L.check(rc, "edt_slerp_merge_speculative")


def test_population_kernels_edges(dev, ops):
    """Population entry points: empty arenas are a no-op, more children than one launch takes is
    refused by the C ABI (the Python layers fall back to per-child calls), an output that is
    also an input is refused."""
    from evolutionarydistributedtraining_amd import EdtError
    from evolutionarydistributedtraining_amd import _lib as L
    bf = torch.bfloat16
    e = torch.empty(0, dtype=bf, device=dev)
    ops.pair_merge_population([{"b1": e, "b2": e, "m1": e, "m2": e, "out": e, "momentum": None,
                                "momentum_in": None, "has_momentum": False}], 0.7, 0.0, False)
    x = [torch.randn(64, device=dev).to(bf) for _ in range(4)]
    ch = lambda out: {"b1": x[0], "b2": x[1], "m1": x[2], "m2": x[3], "out": out, "momentum": None,
                      "momentum_in": None, "has_momentum": False}
    with pytest.raises(EdtError):                    # 17 children: beyond one launch
        ops.pair_merge_population([ch(torch.empty(64, dtype=bf, device=dev)) for _ in range(17)], 0.7, 0.0, False)
    with pytest.raises(EdtError):                    # output == a parent
        ops.pair_merge_population([ch(x[0])], 0.7, 0.0, False)
    with pytest.raises(EdtError):                    # two children writing one buffer
        o = torch.empty(64, dtype=bf, device=dev)
        ops.pair_merge_population([ch(o), ch(o)], 0.7, 0.0, False)
    plan = ops.make_slerp_plan([0, 64], dev)
    t = torch.full((1,), 0.5, dtype=torch.float64, device=dev)
    with pytest.raises(EdtError):                    # Gram form: at most 8 members
        ops.slerp_population(plan, [x[0]] * 9, [(0, 1)], [torch.empty(64, dtype=bf, device=dev)], t, speculate=False)
    with pytest.raises(EdtError):                    # speculative C entry refuses an output over a member
        flat = (L.ctypes.c_int32 * 2)(0, 1)
        L.check(L.lib().edt_slerp_population_speculative(
            L.ptr_array(x[:2]), 2, 1, flat, 1, L.ptr_array([x[0]]), 1, L.ptr(plan.chunks), plan.nchunks,
            L.ptr(plan.seg_first), 1, L.ptr(t), 0.9995, 1e-8, L.ptr(torch.empty(3 * plan.nchunks, dtype=torch.float64,
                                                                                 device=dev)),
            L.ptr(plan.coef), None, L.ptr(torch.empty(1, dtype=torch.int32, device=dev)), 64, L.stream_ptr(dev)),
            "edt_slerp_population_speculative")
    with pytest.raises(EdtError):                    # and so does the Gram form (output == member)
        ops.slerp_population(plan, x[1:3], [(0, 1)], [x[1]], t)
    ops.slerp_population(plan, x[1:3], [(0, 1)], [x[0]], t)  # a separate output is fine
    torch.cuda.synchronize()


def test_errors_are_raised(dev, ops):
    from evolutionarydistributedtraining_amd import EdtError
    th = torch.zeros(16, device=dev)
    with pytest.raises(EdtError):
        ops.outer_step(th, [], None, False, 0.7, 0.0, False)
    with pytest.raises(EdtError):
        ops.outer_step(th, [torch.zeros(15, device=dev)], None, False, 0.7, 0.0, False)
    with pytest.raises(EdtError):   # a worker of the wrong size anywhere in a chained population
        ops.outer_step(th, [torch.zeros(16, device=dev)] * 40 + [torch.zeros(15, device=dev)], None, False,
                       0.7, 0.0, False)
    with pytest.raises(EdtError):   # bf16 master with fp32 workers is not a torch-promotable pair
        ops.outer_step(th.bfloat16(), [torch.zeros(16, device=dev)], None, False, 0.7, 0.0, False)
    with pytest.raises(EdtError):   # host tensors are refused: no CPU path
        ops.outer_step(torch.zeros(16), [torch.zeros(16)], None, False, 0.7, 0.0, False)


def test_c_consumer_runs():
    """The plain-C consumer of include/edt_sync.h (tests/c_abi/abi_consumer.c, built by build()):
    hipMalloc'd buffers, two edt_outer_step calls on the null stream, bit-exact against the C
    oracle, and the negative-code + edt_last_error() convention for a bad argument; then the
    tensor-list SLERP (two-pass and speculative) over separate hipMalloc'd tensors, bit-exact with
    the oracle's lerp branch and with each other; then a resident population of 8 children over 6
    members (r5): the one-pass form and the sharded needed-sums stages (table, sums over two chunk
    ranges, coefficients, blends), every child bit-identical to edt_slerp_merge."""
    import subprocess
    exe = os.path.join(ROOT, "tests", "c_abi", "_build", "abi_consumer")
    if not os.path.exists(exe):
        subprocess.run(["make", "-s", "-C", os.path.dirname(os.path.dirname(exe))], check=True)
    r = subprocess.run([exe], capture_output=True, text=True, timeout=120, cwd="/")
    assert r.returncode == 0, r.stdout + r.stderr
    assert "abi consumer ok" in r.stdout and "slerp list" in r.stdout and "population (8 children" in r.stdout


def test_c_comm_consumer_runs():
    """The plain-C multi-GPU master over include/edt_comm.h (tests/c_abi/comm_consumer.c) at world
    size 1: unique id, init, two outer steps with each of the three sharded schedules (reduce,
    reduce_ordered, exact) bit-exact against the C oracle, then the abort path."""
    import subprocess
    exe = os.path.join(ROOT, "tests", "c_abi", "_build", "comm_consumer")
    if not os.path.exists(exe):
        subprocess.run(["make", "-s", "-C", os.path.dirname(os.path.dirname(exe))], check=True)
    r = subprocess.run([exe], capture_output=True, text=True, timeout=120, cwd="/")
    assert r.returncode == 0, r.stdout + r.stderr
    assert "comm consumer ok" in r.stdout
    for name in ("reduce", "reduce_ordered", "exact"):
        assert f"{name}: bit-exact with the oracle" in r.stdout


# ------------------------------------------------------------------------------------------
# torch CPU scalar-tail emulation (edt_outer_step_tail / edt_pair_merge_tail): with the reference
# host's tail elements, the bf16 regime is bit-exact with the reference on EVERY element

def _tail_bits(numels, dev, threads=1, vec=32):
    from evolutionarydistributedtraining_amd.torchcompat import torch_cpu_tail_bits
    return torch_cpu_tail_bits(numels, vec_elems=vec, num_threads=threads, device=dev)


@pytest.mark.parametrize("idx", range(len(_M["diloco"])))
def test_diloco_golden_bit_exact_with_tails(golden, dev, ops, idx):
    c = golden.diloco_cases()[idx]
    T = len(c["shapes"])
    numels = [int(torch.Size(s).numel()) for s in c["shapes"]]
    tb = _tail_bits(numels, dev)
    prev_buf = None
    for step in c["steps"]:
        pre = step["prefix"]
        theta = flat(golden.tlist("diloco", f"{pre}/base", T)).contiguous()
        workers = [flat(golden.tlist("diloco", f"{pre}/worker{k}", T)).contiguous() for k in range(c["K"])]
        mu = c["momentum"]
        mom = None if mu == 0 else (torch.zeros_like(theta) if prev_buf is None else prev_buf.clone())
        has = mu != 0 and prev_buf is not None
        th_d, mom_d = theta.to(dev), None if mom is None else mom.to(dev)
        ops.outer_step(th_d, [w.to(dev) for w in workers], mom_d, has, c["lr"], mu, c["nesterov"], tail_bits=tb)
        want = flat(golden.tlist("diloco", f"{pre}/out_theta", T))
        assert torch.equal(bits(th_d.cpu()), bits(want)), pre           # every element, every regime
        if step["has_out_buf"]:
            prev_buf = mom_d.cpu()
            assert torch.equal(bits(prev_buf), bits(flat(golden.tlist("diloco", f"{pre}/out_buf", T))))


def test_diloco_large_golden_bit_exact_with_parallel_tails(golden, dev, ops):
    """The golden case whose tensors exceed torch's parallel grain, generated with torch's thread
    count of the generating host: a tail at the end of every parallel chunk, reproduced exactly."""
    c = golden.manifest["diloco_large"]
    T = len(c["shapes"])
    numels = [int(torch.Size(s).numel()) for s in c["shapes"]]
    tb = _tail_bits(numels, dev, threads=c["torch_num_threads"])
    pre = c["name"]
    theta = flat(golden.tlist("diloco", f"{pre}/s0/base", T)).contiguous().to(dev)
    mom = torch.zeros_like(theta)
    for step in (0, 1):
        ws = [flat(golden.tlist("diloco", f"{pre}/s{step}/worker{k}", T)).contiguous().to(dev) for k in range(c["K"])]
        ops.outer_step(theta, ws, mom, step == 1, c["lr"], c["momentum"], c["nesterov"], tail_bits=tb)
        assert torch.equal(bits(theta.cpu()), bits(flat(golden.tlist("diloco", f"{pre}/s{step}/out_theta", T)))), step
    assert torch.equal(bits(mom.cpu()), bits(flat(golden.tlist("diloco", f"{pre}/s1/out_buf", T))))


@pytest.mark.parametrize("idx", range(len(_M["pair_merge"])))
def test_pair_merge_golden_bit_exact_with_tails(golden, dev, ops, idx):
    from tests.test_oracle_golden import pair_inputs
    c = golden.pair_cases()[idx]
    p = pair_inputs(golden, c)
    tb = _tail_bits([int(torch.Size(s).numel()) for s in c["shapes"]], dev)
    n = p["b1"].numel()
    out_d = torch.empty(n, dtype=p["bdt"], device=dev)
    mom_d = None if p["mom"] is None else p["mom"].to(dev)
    ops.pair_merge(p["b1"].to(dev), p["b2"].to(dev), p["m1"].to(dev), p["m2"].to(dev), out_d, mom_d,
                   p["has"], p["lr"], p["mu"], p["nesterov"], tail_bits=tb)
    assert torch.equal(bits(out_d.cpu()), bits(p["want_theta"])), c["name"]
    if p["want_buf"] is not None:
        assert torch.equal(bits(mom_d.cpu()), bits(p["want_buf"].to(p["bdt"])))


@pytest.mark.parametrize("threads,vec", [(1, 32), (3, 32), (8, 16), (16, 32)])
def test_tail_emulation_vs_oracle(oracle, dev, ops, threads, vec):
    """Random bf16 layouts (odd sizes, tensors above the parallel grain): the kernels with a host's
    tail bits equal the oracle with the same host's tail mask, bit for bit; vector and scalar
    (misaligned) bodies."""
    from evolutionarydistributedtraining_amd.torchcompat import torch_cpu_tail_bits
    numels = [70_001, 5, 31, 257 * 160, 33, 100_003]
    n = sum(numels)
    mask = oracle.torch_cpu_tail_mask(numels, vec_elems=vec, num_threads=threads)
    tb = torch_cpu_tail_bits(numels, vec_elems=vec, num_threads=threads, device=dev)
    g = torch.Generator().manual_seed(threads * 100 + vec)
    theta = (torch.randn(n, generator=g) * 0.02).bfloat16()
    ws = [(theta.float() + torch.randn(n, generator=g) * 1e-3).bfloat16() for _ in range(3)]
    mom = (torch.randn(n, generator=g) * 1e-3).bfloat16()
    th_d, m_d = theta.to(dev), mom.to(dev)
    ops.outer_step(th_d, [w.to(dev) for w in ws], m_d, True, 0.7, 0.9, True, tail_bits=tb)
    th, m = theta.clone(), mom.clone()
    oracle.outer_step(th, ws, m, True, 0.7, 0.9, True, mask)
    assert torch.equal(bits(th_d.cpu()), bits(th)) and torch.equal(bits(m_d.cpu()), bits(m))
    assert int(mask.sum()) > 0
    # pair merge, bases merged in the kernel (b2 given)
    out_d = torch.empty(n, dtype=torch.bfloat16, device=dev)
    mom2_d = mom.to(dev)
    ops.pair_merge(ws[0].to(dev), ws[1].to(dev), ws[2].to(dev), theta.to(dev), out_d, mom2_d, True, 0.7, 0.9, True,
                   tail_bits=tb)
    out = torch.empty(n, dtype=torch.bfloat16)
    m2 = mom.clone()
    oracle.pair_merge(ws[0], ws[1], ws[2], theta, out, m2, True, 0.7, 0.9, True, tail=mask)
    assert torch.equal(bits(out_d.cpu()), bits(out)) and torch.equal(bits(mom2_d.cpu()), bits(m2))


@pytest.mark.parametrize("gdt", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("nacc,off", [(1, 0), (3, 0), (8, 1)])
def test_sgd_apply_sum_vs_oracle(oracle, dev, ops, gdt, nacc, off):
    """edt_sgd_apply_sum (reduce_ordered's per-shard step): the partials summed in the given order
    in fp32, then the oracle's SGD from that sum, bit for bit; vector and scalar (misaligned) bodies."""
    n = 50_003
    g = torch.Generator().manual_seed(nacc + off)
    theta = (torch.randn(n + off, generator=g) * 0.02).to(gdt)
    mom = (torch.randn(n + off, generator=g) * 1e-3).to(gdt)
    accs = [torch.randn(n + off, generator=g) * 1e-4 for _ in range(nacc)]
    th_d, m_d = theta.to(dev)[off:], mom.to(dev)[off:]
    ops.sgd_apply_sum(th_d, [a.to(dev)[off:] for a in accs], m_d, True, 0.7, 0.9, True)
    total = accs[0][off:].clone()
    for a in accs[1:]:
        total.add_(a[off:])
    th, m = theta[off:].clone(), mom[off:].clone()
    oracle.sgd_apply(th, total, m, True, 0.7, 0.9, True)
    assert torch.equal(bits(th_d.cpu()), bits(th)) and torch.equal(bits(m_d.cpu()), bits(m))
