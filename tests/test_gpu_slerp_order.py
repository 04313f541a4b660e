"""The SLERP chunk sums follow the documented canonical order bit for bit (edt_slerp.hip "the chunk
sums' canonical order"), in every kernel form: the two-pass stats pass, the
speculative pass, the Gram pass — checked against oracle.canonical_chunk_sums, a numpy
restatement of that order. This pins the cross-lane reduction (permlane swaps + DPP, the values
transposed at levels 32 / 16) to the xor butterfly it restates, on layouts whose segments start
unaligned (head / tail elements), end mid-tile and mid-chunk, and reach the 64 Ki chunk size."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

SIZES = [1, 7, 13, 515, 4093, 65536, 65537, 131077, 200003, 8005]


@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.skip("needs a HIP device")
    return torch.device("cuda:0")


def _layout():
    offs = [0]
    for n in SIZES:
        offs.append(offs[-1] + n)
    return offs


def _members(dt, k, n, seed=5):
    g = torch.Generator().manual_seed(seed)
    base = torch.randn(n, generator=g)
    return [(base + 0.3 * torch.randn(n, generator=g) * (i + 1)).to(dt) for i in range(k)]


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
def test_stats_and_speculative_sums_in_canonical_order(oracle, dev, dt):
    from evolutionarydistributedtraining_amd import _lib as L
    from evolutionarydistributedtraining_amd import ops
    offs = _layout()
    a, b = _members(dt, 2, offs[-1])
    plan = ops.make_slerp_plan(offs, dev)
    want = oracle.canonical_chunk_sums(a, b, plan.chunks_host)
    v0, v1 = a.to(dev), b.to(dev)
    lib, st = L.lib(), L.stream_ptr(dev)
    L.check(lib.edt_slerp_stats(L.ptr(v0), L.ptr(v1), L.dtype_code(v0), L.ptr(plan.chunks), plan.nchunks,
                                L.ptr(plan.partial), st), "edt_slerp_stats")
    got = plan.partial[:3 * plan.nchunks].view(-1, 3).cpu().numpy()
    assert np.array_equal(got.view(np.int64), want.view(np.int64)), np.abs(got - want).max()
    out = torch.empty_like(v0)
    t = torch.full((plan.nseg,), 0.4, dtype=torch.float64, device=dev)
    plan.partial.zero_()
    ops.slerp_arena(plan, v0, v1, out, t, speculate=True)
    got = plan.partial[:3 * plan.nchunks].view(-1, 3).cpu().numpy()
    assert np.array_equal(got.view(np.int64), want.view(np.int64)), np.abs(got - want).max()


@pytest.mark.parametrize("M", [1, 3, 8])
@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
def test_gram_sums_in_canonical_order(oracle, dev, M, dt):
    from evolutionarydistributedtraining_amd import ops
    offs = _layout()
    mem = _members(dt, M, offs[-1], seed=11 + M)
    plan = ops.make_slerp_plan(offs, dev)
    gram = ops.slerp_gram([m.to(dev) for m in mem], plan.chunks, plan.nchunks).cpu().numpy()
    col = 0
    for i in range(M):
        for j in range(i, M):
            want = oracle.canonical_chunk_sums(mem[i], mem[j], plan.chunks_host)[:, 2]
            assert np.array_equal(gram[:, col].view(np.int64), want.view(np.int64)), (i, j)
            col += 1


def test_gram_rows_are_owned_by_the_caller(dev):
    """without `gram`, slerp_gram's rows come back in a tensor the caller owns — the
    stream's pooled scratch the pass ran in is reused by the next SLERP call, which must leave the
    returned rows untouched."""
    from evolutionarydistributedtraining_amd import ops
    offs = _layout()
    mem = [m.to(dev) for m in _members(torch.bfloat16, 4, offs[-1], seed=23)]
    plan = ops.make_slerp_plan(offs, dev)
    gram = ops.slerp_gram(mem, plan.chunks, plan.nchunks)
    keep = gram.clone()
    t = torch.full((plan.nseg,), 0.4, dtype=torch.float64, device=dev)
    outs = [torch.empty_like(mem[0]) for _ in range(3)]
    ops.slerp_population(plan, [m.flip(0).contiguous() for m in mem], [(0, 1), (1, 2), (3, 0)], outs, t,
                         speculate=False)
    ops.slerp_gram([m * 2 for m in mem], plan.chunks, plan.nchunks)
    torch.cuda.synchronize()
    assert torch.equal(gram.view(torch.int64), keep.view(torch.int64))
