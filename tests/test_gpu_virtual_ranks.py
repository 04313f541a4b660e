"""The HIP kernels inside the N-rank multi-GPU schedules, on one MI355X: N virtual ranks in one
process (collectives.VirtualWorld; one thread per rank, collectives as device copies / fp32 sums
on the shared stream, RCCL's in-place conventions). This runs on the device exactly what each
rank issues at N = 2 / 4 / 8 — the in-place reduce-scatter offsets, the all-to-all
[dest rank][shard] layout, the all-gather into the worker arenas, shards that cross bucket and
tensor ends, the n_pad tail — which the world-1 RCCL runs cannot (every collective is an
identity there).

  exact/theta, exact/workers: bit-exact with the single-GPU fused step over the whole population
  reduce/theta:               bit-exact with the oracle's partial/SGD split summed in rank order
                              (the virtual ranks' order), and within DESIGN §3's reassociation
                              bound of the reference's sequential order
  PopulationCrossover:        every child bit-identical to the single-GPU kernel on its parents
"""
import pytest
import torch

from evolutionarydistributedtraining_amd import ops
from evolutionarydistributedtraining_amd.collectives import VirtualWorld
from tests.virtual_schedules import bits, population, reduce_reference, reduce_tol, run_sharded

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0")
# 292,187 elements: tensors of odd sizes so shards cross tensor ends; with a bucket of 37 units
# (unit = N x 64 elements) the buckets end mid-tensor and the last one is ragged up to n_pad
SHAPES = [(37, 11), (5,), (1,), (256, 513), (129,), (3, 9001), (1001,), (2, 77)]


def _fused(theta, gens):
    th = theta.clone()
    mom = torch.zeros_like(th)
    for i, ws in enumerate(gens):
        ops.outer_step(th, ws, mom, i > 0, 0.7, 0.9, True)
    torch.cuda.synchronize()
    return th, mom


@pytest.mark.parametrize("world", [2, 4, 8])
@pytest.mark.parametrize("mode,broadcast", [("exact", "theta"), ("exact", "workers"), ("reduce", "theta"),
                                            ("reduce_ordered", "theta")])
@pytest.mark.parametrize("tdt,wdt", [(torch.float32, torch.float32), (torch.float32, torch.bfloat16),
                                     (torch.bfloat16, torch.bfloat16)])
def test_sharded_schedule_on_virtual_ranks(oracle, world, mode, broadcast, tdt, wdt):
    layout, theta, gens = population(SHAPES, tdt, wdt, 8, steps=2, device=DEV)
    res = run_sharded(world, layout, tdt, wdt, theta, gens, DEV, mode=mode, broadcast=broadcast,
                      bucket_elems=world * 64 * 37)
    torch.cuda.synchronize()
    n = layout.total
    assert len(res[0]["buckets"]) >= 3 and res[0]["n_pad"] > n
    assert (res[0]["mode"], res[0]["broadcast"]) == (mode, broadcast)
    for r in res:
        assert torch.equal(bits(r["theta"]), bits(res[0]["theta"]))
    got, mom = res[0]["theta"][:n], res[0]["mom"]
    if mode == "exact":
        th_f, mom_f = _fused(theta, gens)
        assert torch.equal(bits(got), bits(th_f))
        assert torch.equal(bits(mom), bits(mom_f))
        if broadcast == "workers":
            want = th_f.to(wdt)
            for r in res:
                for w in r["workers"]:
                    assert torch.equal(bits(w[:n]), bits(want))
    else:
        cpu_gens = [[w.cpu() for w in ws] for ws in gens]
        th_rs, mom_rs = reduce_reference(oracle, theta.cpu(), cpu_gens, world)
        assert torch.equal(bits(got.cpu()), bits(th_rs))
        assert torch.equal(bits(mom.cpu()), bits(mom_rs))
        th_ref = theta.cpu().clone()
        mom_ref = torch.zeros_like(th_ref)
        for i, ws in enumerate(cpu_gens):
            oracle.outer_step(th_ref, ws, mom_ref, i > 0, 0.7, 0.9, True)
        tol = reduce_tol(th_ref, mom_ref, tdt, gens=cpu_gens)
        assert ((got.cpu().float() - th_ref.float()).abs() <= tol).all()


@pytest.mark.parametrize("world", [2, 4, 8])
def test_population_crossover_on_virtual_ranks(world):
    """PopulationCrossover (one member per rank, grouped p2p of each child's parents) with the
    HIP SLERP and pair-merge kernels: every child equals the single-GPU kernel on its parents."""
    from evolutionarydistributedtraining_amd.distributed import PopulationCrossover
    from evolutionarydistributedtraining_amd.params import ParamLayout
    layout = ParamLayout([(33, 7), (5,), (3000,), (1,), (64, 65)])
    n = layout.total
    g = torch.Generator().manual_seed(5)
    base = [(torch.randn(n, generator=g) * 0.02).bfloat16().to(DEV) for _ in range(world)]
    trained = [(b.float() + torch.randn(n, generator=g).to(DEV) * 1e-3).bfloat16() for b in base]
    mom = [(torch.randn(n, generator=g) * 1e-3).bfloat16().to(DEV) for _ in range(world)]
    pairs = [((c * 3 + 1) % world, (c * 5 + 2) % world) for c in range(world)]
    t = torch.tensor([0.3, 0.5, 0.9, 0.5, 0.43], dtype=torch.float64, device=DEV)

    def body(comm):
        r = comm.rank
        pc = PopulationCrossover(layout, torch.bfloat16, DEV, comm=comm)
        s_out = torch.empty(n, dtype=torch.float32, device=DEV)
        pc.slerp_step(trained[r], pairs, t, s_out)
        child = torch.empty(n, dtype=torch.bfloat16, device=DEV)
        cmom = torch.empty(n, dtype=torch.bfloat16, device=DEV)
        pc.pair_merge_step(base[r], trained[r], mom[r], pairs, child, cmom, generation=1)
        return s_out, child, cmom

    res = VirtualWorld(world).run(body)
    torch.cuda.synchronize()
    plan = ops.make_slerp_plan(layout.offsets, DEV)
    for c, (i, j) in enumerate(pairs):
        want = torch.empty(n, dtype=torch.float32, device=DEV)
        ops.slerp_arena(plan, trained[i], trained[j], want, t, speculate=False)
        out = torch.empty(n, dtype=torch.bfloat16, device=DEV)
        m_out = torch.empty_like(out)
        ops.pair_merge(base[i], base[j], trained[i], trained[j], out, m_out, True, 0.7, 0.9, True,
                       momentum_in=mom[i])
        torch.cuda.synchronize()
        assert torch.equal(res[c][0].view(torch.int32), want.view(torch.int32)), c
        assert torch.equal(res[c][1].view(torch.int16), out.view(torch.int16)), c
        assert torch.equal(res[c][2].view(torch.int16), m_out.view(torch.int16)), c


@pytest.mark.parametrize("world", [2, 4, 8])
@pytest.mark.parametrize("out_dt", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("groups", [1, 3])
def test_sharded_population_slerp_on_virtual_ranks(world, out_dt, groups):
    """The link-balanced population SLERP (each rank: a range of whole chunks of all members, Gram
    rows all-gathered, its range of every child blended and sent to the child's rank) with the HIP
    passes: every child bit-identical to edt_slerp_merge on its two parents, and the dots too."""
    from evolutionarydistributedtraining_amd.distributed import ShardedPopulationCrossover
    from evolutionarydistributedtraining_amd.params import ParamLayout
    layout = ParamLayout([(513, 301), (7,), (1,), (131073,), (3, 1001), (64, 2049), (5,), (300_007,)])
    n = layout.total
    g = torch.Generator().manual_seed(8)
    base = torch.randn(n, generator=g) * 0.02
    members = [(base + torch.randn(n, generator=g) * 0.02 * (0.005 if r % 3 else 0.1)).bfloat16().to(DEV)
               for r in range(world)]
    pairs = [((3 * c + 1) % world, (5 * c + 2) % world) for c in range(world)]
    t = torch.tensor([0.3, 0.5, 0.9, 0.5, 0.43, 0.7, 0.5, 0.6], dtype=torch.float64, device=DEV)

    def body(comm):
        sp = ShardedPopulationCrossover(layout, torch.bfloat16, DEV, kind="slerp", out_dtype=out_dt, comm=comm,
                                        groups=groups)
        out = torch.full((n,), float("nan"), dtype=out_dt, device=DEV)
        dots = sp.slerp_step(members[comm.rank], pairs, t, out)
        return out, dots.clone()

    res = VirtualWorld(world).run(body)
    torch.cuda.synchronize()
    plan = ops.make_slerp_plan(layout.offsets, DEV)
    for c, (i, j) in enumerate(pairs):
        want = torch.empty(n, dtype=out_dt, device=DEV)
        ops.slerp_arena(plan, members[i], members[j], want, t, speculate=False)
        torch.cuda.synchronize()
        assert torch.equal(bits(res[c][0]), bits(want)), c
        assert torch.equal(res[0][1][c], plan.dots[:plan.nseg]), c


@pytest.mark.parametrize("world", [2, 3, 4, 5, 8])
@pytest.mark.parametrize("gen", range(4))
def test_sharded_population_roulette_graphs_on_virtual_ranks(world, gen):
    """r5: the sharded population forms only the needed sums (edt_slerp_needed_sums over each rank's
    chunk range, those table rows all-gathered) on pair graphs drawn by EDT_RL's roulette selection
    (schedule.roulette_generation_pairs: world pairs over world members, hubs and repeated pairs):
    every child bit-identical to edt_slerp_merge on its two parents, dots too, with 1 and 3 groups."""
    from evolutionarydistributedtraining_amd.distributed import ShardedPopulationCrossover
    from evolutionarydistributedtraining_amd.params import ParamLayout
    from evolutionarydistributedtraining_amd.schedule import roulette_generation_pairs
    layout = ParamLayout([(257, 301), (7,), (1,), (65537,), (3, 1001), (5,), (200_003,)])
    n = layout.total
    pairs = [tuple(p) for p in roulette_generation_pairs(world, gen + 1, seed=77)[gen]["pairs"]]
    g = torch.Generator().manual_seed(10 + gen)
    base = torch.randn(n, generator=g) * 0.02
    members = [(base + torch.randn(n, generator=g) * 0.02 * (0.005 if r % 3 else 0.1)).bfloat16().to(DEV)
               for r in range(world)]
    t = torch.tensor([0.3, 0.5, 0.9, 0.5, 0.43, 0.7, 0.6], dtype=torch.float64, device=DEV)
    lay = ops.needed_table(pairs, world, ops.make_slerp_plan(layout.offsets, DEV).nchunks)
    assert sum(nt for _, nt in lay.blocks) <= world * (world + 1) // 2
    plan = ops.make_slerp_plan(layout.offsets, DEV)
    for groups in (1, 3):
        def body(comm):
            sp = ShardedPopulationCrossover(layout, torch.bfloat16, DEV, kind="slerp", out_dtype=torch.bfloat16,
                                            comm=comm, groups=groups)
            out = torch.full((n,), float("nan"), dtype=torch.bfloat16, device=DEV)
            dots = sp.slerp_step(members[comm.rank], pairs, t, out)
            return out, dots.clone()

        res = VirtualWorld(world).run(body)
        torch.cuda.synchronize()
        for c, (i, j) in enumerate(pairs):
            want = torch.empty(n, dtype=torch.bfloat16, device=DEV)
            ops.slerp_arena(plan, members[i], members[j], want, t, speculate=False)
            torch.cuda.synchronize()
            assert torch.equal(bits(res[c][0]), bits(want)), (groups, c, pairs)
            assert torch.equal(res[0][1][c], plan.dots[:plan.nseg]), (groups, c)


def test_sharded_population_dense_graph_takes_the_triangle_layout():
    """r6: a pair graph past the chord slots (a hub in 7 of the 8 pairs) puts its component on the
    triangle layout of the needed-sums pass; through the shards (world 8, the table rows of every
    rank's chunk range all-gathered, 1 and 3 groups) every child and its dots stay bit-identical to
    edt_slerp_merge on its two parents."""
    from evolutionarydistributedtraining_amd.distributed import ShardedPopulationCrossover
    from evolutionarydistributedtraining_amd.params import ParamLayout
    world = 8
    layout = ParamLayout([(257, 301), (7,), (1,), (65537,), (3, 1001), (5,), (200_003,)])
    n = layout.total
    pairs = [(0, m) for m in range(1, 8)] + [(1, 2)]
    assert [c["stats_layout"] for c in ops.population_layout(pairs, world, False)["components"]] == ["triangle"]
    g = torch.Generator().manual_seed(21)
    base = torch.randn(n, generator=g) * 0.02
    members = [(base + torch.randn(n, generator=g) * 0.02 * (0.005 if r % 2 else 0.5)).bfloat16().to(DEV)
               for r in range(world)]
    t = torch.tensor([0.3, 0.5, 0.9, 0.5, 0.43, 0.7, 0.6], dtype=torch.float64, device=DEV)
    plan = ops.make_slerp_plan(layout.offsets, DEV)
    for groups in (1, 3):
        def body(comm):
            sp = ShardedPopulationCrossover(layout, torch.bfloat16, DEV, kind="slerp", out_dtype=torch.bfloat16,
                                            comm=comm, groups=groups)
            out = torch.full((n,), float("nan"), dtype=torch.bfloat16, device=DEV)
            dots = sp.slerp_step(members[comm.rank], pairs, t, out)
            return out, dots.clone()

        res = VirtualWorld(world).run(body)
        torch.cuda.synchronize()
        for c, (i, j) in enumerate(pairs):
            want = torch.empty(n, dtype=torch.bfloat16, device=DEV)
            ops.slerp_arena(plan, members[i], members[j], want, t, speculate=False)
            torch.cuda.synchronize()
            assert torch.equal(bits(res[c][0]), bits(want)), (groups, c)
            assert torch.equal(res[0][1][c], plan.dots[:plan.nseg]), (groups, c)


def test_needed_sums_entries_match_the_population_pass():
    """edt_slerp_needed_sums over a chunk range (row0 > 0, a chunk table relative to a shard) writes
    the same rows as the whole-table call, and edt_slerp_needed_coef gives edt_slerp_population's
    coefficients and dots."""
    from evolutionarydistributedtraining_amd.schedule import roulette_generation_pairs
    sizes = [70_001, 9, 131_072, 4099, 1]
    offs = [0]
    for x in sizes:
        offs.append(offs[-1] + x)
    g = torch.Generator().manual_seed(3)
    base = torch.randn(offs[-1], generator=g) * 0.02
    mem = [(base + torch.randn(offs[-1], generator=g) * 1e-3).bfloat16().to(DEV) for _ in range(8)]
    pairs = [tuple(p) for p in roulette_generation_pairs(8, 1, seed=5)[0]["pairs"]]
    plan = ops.make_slerp_plan(offs, DEV, chunk_elems=8192)
    lay = ops.needed_table(pairs, 8, plan.nchunks)
    whole = torch.full((lay.doubles,), float("nan"), dtype=torch.float64, device=DEV)
    ops.slerp_needed_sums(mem, lay, plan.chunks, plan.nchunks, whole, 0)
    part = torch.full_like(whole, float("nan"))
    cut = plan.nchunks // 3
    base_el = int(plan.chunks_host[cut, 0]) // 8 * 8
    shard = [m[base_el:].contiguous() for m in mem]
    loc = plan.chunks[cut:].clone()
    loc[:, 0] -= base_el
    ops.slerp_needed_sums(mem, lay, plan.chunks[:cut], cut, part, 0)
    ops.slerp_needed_sums(shard, lay, loc, plan.nchunks - cut, part, cut)
    torch.cuda.synchronize()
    assert torch.equal(whole.view(torch.int64), part.view(torch.int64))
    t = torch.full((plan.nseg,), 0.4, dtype=torch.float64, device=DEV)
    coef, dots = ops.slerp_needed_coef(plan, whole, lay, t)
    outs = [torch.empty(offs[-1], dtype=torch.bfloat16, device=DEV) for _ in pairs]
    want_dots = ops.slerp_population(plan, mem, pairs, outs, t, speculate=False).clone()
    torch.cuda.synchronize()
    assert torch.equal(dots[:len(pairs), :plan.nseg].cpu(), want_dots[:len(pairs), :plan.nseg].cpu())


@pytest.mark.parametrize("world", [2, 8])
def test_sharded_population_pair_merge_on_virtual_ranks(world):
    """EDT-LM children through the shards (edt_pair_merge_population on every rank's range) equal
    edt_pair_merge per child on whole parents, child and momentum."""
    from evolutionarydistributedtraining_amd.distributed import ShardedPopulationCrossover
    from evolutionarydistributedtraining_amd.params import ParamLayout
    layout = ParamLayout([(513, 301), (7,), (131073,), (5,)])
    n = layout.total
    g = torch.Generator().manual_seed(9)
    base = [(torch.randn(n, generator=g) * 0.02).bfloat16().to(DEV) for _ in range(world)]
    trained = [(b.float() + torch.randn(n, generator=g).to(DEV) * 1e-3).bfloat16() for b in base]
    mom = [(torch.randn(n, generator=g) * 1e-3).bfloat16().to(DEV) for _ in range(world)]
    pairs = [((3 * c + 1) % world, (5 * c + 2) % world) for c in range(world)]

    def body(comm):
        r = comm.rank
        sp = ShardedPopulationCrossover(layout, torch.bfloat16, DEV, kind="sgd", comm=comm)
        out, out_m = torch.empty(n, dtype=torch.bfloat16, device=DEV), torch.empty(n, dtype=torch.bfloat16, device=DEV)
        sp.pair_merge_step(base[r], trained[r], mom[r], pairs, out, out_m, generation=1)
        return out, out_m

    res = VirtualWorld(world).run(body)
    torch.cuda.synchronize()
    for c, (i, j) in enumerate(pairs):
        out, m_out = torch.empty(n, dtype=torch.bfloat16, device=DEV), torch.empty(n, dtype=torch.bfloat16, device=DEV)
        ops.pair_merge(base[i], base[j], trained[i], trained[j], out, m_out, True, 0.7, 0.9, True, momentum_in=mom[i])
        torch.cuda.synchronize()
        assert torch.equal(bits(res[c][0]), bits(out)), c
        assert torch.equal(bits(res[c][1]), bits(m_out)), c


def test_bench_population_measurement_on_virtual_ranks():
    """bench.py's N > 1 configs[4] measurement (bench_population) runs its schedule end to end
    through a communicator: here 4 virtual ranks on the 125M layout (the driver's 8-GPU run uses
    RCCL and the 7B body)."""
    import types

    import bench
    args = types.SimpleNamespace(steps=4, population_groups=4)
    res = VirtualWorld(4).run(lambda comm: bench.bench_population(args, bench.Runtime(DEV), comm,
                                                                  layout_name="gpt2_small"))
    for r in res:
        assert r["sharded"]["ms"] > 0 and r["per_child"]["ms"] > 0
        assert r["sharded_pipelined"]["ms"] > 0 and r["sharded_pipelined"]["groups"] == 4
        assert r["sharded"]["wire_bytes_per_rank"] == 2 * 3 * (124439808 * 2 // 4)


@pytest.mark.parametrize("world", [2, 8])
def test_sharded_exact_with_torch_tails(world):
    """exact mode with cpu_tails (the reference host's bf16 scalar tails): every rank's shard step
    takes its slice of the tail bitmask, and the gathered master equals the single-GPU fused step
    with the same bits."""
    from evolutionarydistributedtraining_amd.torchcompat import torch_cpu_tail_bits
    layout, theta, gens = population(SHAPES, torch.bfloat16, torch.bfloat16, 8, steps=2, device=DEV)
    tb = torch_cpu_tail_bits(layout.numels, vec_elems=32, num_threads=8, device=DEV)
    th, mom = theta.clone(), torch.zeros_like(theta)
    for i, ws in enumerate(gens):
        ops.outer_step(th, ws, mom, i > 0, 0.7, 0.9, True, tail_bits=tb)
    from evolutionarydistributedtraining_amd.distributed import ShardedOuterSync
    k_local = 8 // world

    def body(comm):
        s = ShardedOuterSync(layout, torch.bfloat16, torch.bfloat16, k_local, DEV, mode="exact", broadcast="theta",
                             bucket_elems=world * 64 * 37, comm=comm, cpu_tails=(32, 8))
        s.theta.flat.copy_(theta)
        for ws in gens:
            for j, a in enumerate(s.workers):
                a.flat.copy_(ws[comm.rank * k_local + j])
            s.step()
        return s.gather_theta().clone()

    res = VirtualWorld(world).run(body)
    torch.cuda.synchronize()
    for r in res:
        assert torch.equal(bits(r), bits(th))
    plain = theta.clone()
    m2 = torch.zeros_like(theta)
    for i, ws in enumerate(gens):
        ops.outer_step(plain, ws, m2, i > 0, 0.7, 0.9, True)
    assert not torch.equal(bits(plain), bits(th))      # the tails do change bits here
