"""The split SLERP passes of the C ABI (include/edt_sync.h: edt_slerp_stats -> edt_slerp_coef ->
edt_slerp_blend), called one by one the way a host that schedules the passes itself would (e.g.
the stats of the next pair overlapping the blend of this one): the chunk sums, coefficients,
dots and output are bit-identical to the one-call edt_slerp_merge, for every input / output
dtype route, over segments in the lerp branch, the SLERP branch, zero tensors and empty ones —
and the output agrees with the oracle's restatement of EDT_RL/crossover.py:11-43 (lerp branch
bit-exact, SLERP branch within the golden bar of test_gpu_fuzz)."""
import pytest
import torch

from tests.golden_data import bits

pytestmark = pytest.mark.gpu

ROUTES = [(torch.float32, torch.float32), (torch.bfloat16, torch.bfloat16), (torch.bfloat16, torch.float32),
          (torch.float32, torch.bfloat16)]


@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.skip("needs a HIP device")
    return torch.device("cuda:0")


def _inputs(seed):
    """Segments: lerp branch (tiny spread), SLERP branch (far), a zero parent, an empty segment,
    a vector-ragged one, and one longer than a chunk."""
    g = torch.Generator().manual_seed(seed)
    sizes = [5000, 3001, 0, 777, 9, 70000]
    spreads = [1e-4, 0.5, None, 2.0, 0.05, 0.02]
    v0s, v1s = [], []
    for n, sp in zip(sizes, spreads):
        a = torch.randn(n, generator=g) * 0.02
        b = torch.zeros(n) if sp is None else a + torch.randn(n, generator=g) * 0.02 * sp
        v0s.append(a)
        v1s.append(b)
    offs = [0]
    for n in sizes:
        offs.append(offs[-1] + n)
    t = torch.tensor([0.5, 0.3, 0.5, 0.9, 0.1, 0.5], dtype=torch.float64)
    return torch.cat(v0s), torch.cat(v1s), offs, t


@pytest.mark.parametrize("idt,odt", ROUTES)
@pytest.mark.parametrize("seed", [0, 1])
def test_split_passes_equal_one_call_merge(oracle, dev, idt, odt, seed):
    from evolutionarydistributedtraining_amd import _lib as L
    from evolutionarydistributedtraining_amd import ops
    lib = L.lib()
    v0, v1, offs, t = _inputs(seed)
    v0, v1 = v0.to(idt), v1.to(idt)
    n = offs[-1]
    a, b, td = v0.to(dev), v1.to(dev), t.to(dev)
    ic, oc = L.dtype_code(a), L.dtype_code(torch.empty(0, dtype=odt))
    st = L.stream_ptr(dev)

    # one call
    plan1 = ops.make_slerp_plan(offs, dev, chunk_elems=4096)
    out1 = torch.empty(n, dtype=odt, device=dev)
    L.check(lib.edt_slerp_merge(L.ptr(a), L.ptr(b), ic, L.ptr(out1), oc, L.ptr(plan1.chunks), plan1.nchunks,
                                L.ptr(plan1.seg_first), plan1.nseg, L.ptr(td), 0.9995, 1e-8, L.ptr(plan1.partial),
                                L.ptr(plan1.coef), L.ptr(plan1.dots), st), "edt_slerp_merge")
    sums1 = plan1.partial[:3 * plan1.nchunks].clone()     # the workspace is shared per stream
    # the three passes, separately
    plan2 = ops.make_slerp_plan(offs, dev, chunk_elems=4096)
    out2 = torch.empty(n, dtype=odt, device=dev)
    L.check(lib.edt_slerp_stats(L.ptr(a), L.ptr(b), ic, L.ptr(plan2.chunks), plan2.nchunks, L.ptr(plan2.partial),
                                st), "edt_slerp_stats")
    L.check(lib.edt_slerp_coef(L.ptr(plan2.partial), L.ptr(plan2.seg_first), plan2.nseg, L.ptr(td), 0.9995, 1e-8,
                               L.ptr(plan2.coef), L.ptr(plan2.dots), st), "edt_slerp_coef")
    L.check(lib.edt_slerp_blend(L.ptr(a), L.ptr(b), ic, L.ptr(out2), oc, L.ptr(plan2.chunks), plan2.nchunks,
                                L.ptr(plan2.coef), st), "edt_slerp_blend")
    torch.cuda.synchronize()
    nc = 3 * plan1.nchunks
    assert torch.equal(bits(sums1.cpu()), bits(plan2.partial[:nc].cpu()))
    assert torch.equal(bits(plan1.coef.cpu()), bits(plan2.coef.cpu()))
    assert torch.equal(bits(plan1.dots.cpu()), bits(plan2.dots.cpu()))
    assert torch.equal(bits(out1.cpu()), bits(out2.cpu()))

    # against the oracle, per segment (fp32 outputs: the bar is stated on fp32)
    if odt != torch.float32:
        return
    got = out2.cpu()
    for s in range(len(offs) - 1):
        lo, hi = offs[s], offs[s + 1]
        if hi == lo:
            continue
        x, y = v0[lo:hi].float(), v1[lo:hi].float()
        want = oracle.slerp(float(t[s]), x, y).float()
        c0, c1, dot = oracle.slerp_coefficients(float(t[s]), x, y)
        if abs(float(dot)) > 0.9995:
            assert torch.equal(bits(got[lo:hi]), bits(want)), s
        else:
            tol = 4e-6 * (abs(float(c0)) * x.abs() + abs(float(c1)) * y.abs()) + 1e-30
            assert ((got[lo:hi] - want).abs() <= tol).all(), (s, (got[lo:hi] - want).abs().max().item())


def test_split_passes_reject_bad_arguments(dev):
    """The C ABI's error convention on the split passes: a negative code and a message, nothing
    launched (unknown dtype code; negative chunk / segment counts, which would otherwise size a
    grid from a negative number)."""
    from evolutionarydistributedtraining_amd import _lib as L
    from evolutionarydistributedtraining_amd import ops
    lib = L.lib()
    plan = ops.make_slerp_plan([0, 100], dev, chunk_elems=4096)
    a = torch.zeros(100, device=dev)
    t = torch.full((1,), 0.5, dtype=torch.float64, device=dev)
    st = L.stream_ptr(dev)
    P = L.ptr
    assert lib.edt_slerp_stats(P(a), P(a), 99, P(plan.chunks), plan.nchunks, P(plan.partial), st) < 0
    assert b"dtype" in lib.edt_last_error()
    assert lib.edt_slerp_blend(P(a), P(a), 0, P(a), 99, P(plan.chunks), plan.nchunks, P(plan.coef), st) < 0
    assert lib.edt_slerp_stats(P(a), P(a), 0, P(plan.chunks), -1, P(plan.partial), st) < 0
    assert b"negative" in lib.edt_last_error()
    assert lib.edt_slerp_blend(P(a), P(a), 0, P(a), 0, P(plan.chunks), -3, P(plan.coef), st) < 0
    assert lib.edt_slerp_coef(P(plan.partial), P(plan.seg_first), -1, P(t), 0.9995, 1e-8, P(plan.coef), None, st) < 0
    assert b"negative" in lib.edt_last_error()
    assert lib.edt_slerp_merge(P(a), P(a), 0, P(a), 0, P(plan.chunks), -1, P(plan.seg_first), 1, P(t), 0.9995, 1e-8,
                               P(plan.partial), P(plan.coef), None, st) < 0
    torch.cuda.synchronize()
