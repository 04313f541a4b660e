"""The SLERP chunk sums follow the documented canonical order bit for bit (edt_slerp.hip "the chunk
sums' canonical order"), in every kernel form: the two-pass stats pass, the
speculative pass, the population's needed-sums pass in both its layouts (needed / triangle) —
checked against oracle.canonical_chunk_sums, a numpy
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


GRAPHS = {
    "self_pair": (1, [(0, 0)]),
    "ring3": (3, [(0, 1), (1, 2), (2, 0)]),                                  # needed: norms + ring dots
    "chords5": (5, [(0, 1), (1, 2), (2, 3), (3, 4), (4, 0), (0, 2), (1, 3)]),  # needed: ring + 2 chords
    "k5": (5, [(a, b) for a in range(5) for b in range(a + 1, 5)]),           # triangle: 5 chords > 4 slots
    "k8": (8, [(a, b) for a in range(8) for b in range(a + 1, 8)]),           # triangle, every pair
    "star8": (8, [(0, m) for m in range(1, 8)] + [(2, 3)]),                   # triangle, 5 dots masked on
}


@pytest.mark.parametrize("name", sorted(GRAPHS))
@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
def test_population_sums_in_canonical_order(oracle, dev, name, dt):
    """Every column the needed-sums pass forms (edt_slerp_needed_sums over the whole layout: the
    norms, ring dots, chords — or, past the chord slots, the triangle layout's masked dots) equals
    the canonical chunk sums of its two members; unused columns are reported as (-1, -1)."""
    from evolutionarydistributedtraining_amd import ops
    M, pairs = GRAPHS[name]
    offs = _layout()
    mem = _members(dt, M, offs[-1], seed=11 + M)
    plan = ops.make_slerp_plan(offs, dev)
    layout = ops.needed_table(pairs, M, plan.nchunks)
    want_kind = "triangle" if name in ("k5", "k8", "star8") else "needed"
    assert all(c["stats_layout"] == want_kind for c in ops.population_layout(pairs, M, False)["components"])
    table = torch.full((max(1, layout.doubles),), float("nan"), dtype=torch.float64, device=dev)
    ops.slerp_needed_sums([m.to(dev) for m in mem], layout, plan.chunks, plan.nchunks, table, 0)
    table = table.cpu().numpy()
    used = 0
    for b, (off, nt) in enumerate(layout.blocks):
        rows = table[off:off + plan.nchunks * nt].reshape(plan.nchunks, nt)
        for x, (i, j) in enumerate(layout.columns[b]):
            if i < 0:
                continue
            used += 1
            want = oracle.canonical_chunk_sums(mem[i], mem[j], plan.chunks_host)[:, 2]
            assert np.array_equal(rows[:, x].view(np.int64), want.view(np.int64)), (name, b, x, i, j)
    dots = {tuple(sorted(p)) for p in pairs if p[0] != p[1]}
    assert used == len({m for p in pairs for m in p}) + len(dots)    # the norms and the dots used, no more
