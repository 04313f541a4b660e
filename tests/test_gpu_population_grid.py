"""The co-located population passes past the dispatch cap: edt_slerp_population_speculative with
more than 8 distinct parents (the per-child pass, block -> (unit, child)) launches units x children
workgroups, which passes HIP's 2^32 - 1 work-item limit once a member holds more than ~2.1G
elements with 16 children. The launches are split into groups of whole 8-unit XCD groups
(colocated_launches); every child must still be bit-identical to edt_slerp_merge on its two
parents. 9 members + 16 children of 2.2G bf16 elements (110 GB): the lineage form (one pass) and
independent members (the pass + the co-located redo blends)."""
import pytest
import torch

pytestmark = pytest.mark.gpu
BF = torch.bfloat16


@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.skip("needs a HIP device")
    return torch.device("cuda:0")


def _fill(dst, gen, scale, base=None, rel=0.0):
    step = 1 << 28
    for s in range(0, dst.numel(), step):
        e = min(dst.numel(), s + step)
        x = torch.randn(e - s, device=dst.device, generator=gen) * scale
        if base is not None:
            x = base[s:e].float() + x * rel
        dst[s:e] = x.to(dst.dtype)


@pytest.mark.parametrize("lineage", [True, False])
def test_colocated_population_past_the_dispatch_cap(dev, lineage):
    import gc
    from evolutionarydistributedtraining_amd import ops
    gc.collect()
    torch.cuda.empty_cache()
    M, Q = 9, 16
    sizes = [1 << 30, 3 + (1 << 29), 700_000_001, 77]          # 2.22G elements, 4 segments
    offs = [0]
    for n in sizes:
        offs.append(offs[-1] + n)
    P = offs[-1]
    free, _ = torch.cuda.mem_get_info(dev)
    if free < (M + Q + 2) * P * 2 + (8 << 30):
        pytest.skip(f"needs {(M + Q + 2) * P * 2 / 1e9:.0f} GB of HBM")
    gen = torch.Generator(device=dev).manual_seed(9)
    members = [torch.empty(P, dtype=BF, device=dev) for _ in range(M)]
    if lineage:
        base = torch.empty(P, dtype=BF, device=dev)
        _fill(base, gen, 0.02)
        for m in members:
            _fill(m, gen, 0.02, base=base, rel=0.005)
        del base
    else:
        for m in members:
            _fill(m, gen, 0.02)
    plan = ops.make_slerp_plan(offs, dev)
    assert plan.nchunks * 32 * Q > 0xffffffff // 256            # past the cap: several launches
    pairs = [(q % M, (3 * q + 1) % M) for q in range(Q)]
    outs = [torch.empty(P, dtype=BF, device=dev) for _ in range(Q)]
    t = torch.rand(len(sizes), dtype=torch.float64, generator=torch.Generator().manual_seed(9)).to(dev)
    dots = ops.slerp_population(plan, members, pairs, outs, t, speculate=True)
    torch.cuda.synchronize()
    if lineage:
        assert bool((dots.abs() > 0.9995).all())
    want = torch.empty(P, dtype=BF, device=dev)
    for q, (i, j) in enumerate(pairs):
        ops.slerp_arena(plan, members[i], members[j], want, t, speculate=False)
        torch.cuda.synchronize()
        assert torch.equal(outs[q].view(torch.int16), want.view(torch.int16)), (q, i, j)
    del members, outs, want
    gc.collect()
    torch.cuda.empty_cache()
