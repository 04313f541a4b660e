"""Rank-resident EDT generations (population.ResidentPopulation).

The check is a plain restatement of the reference's generation flow, driven by the same seeded
host RNGs: EDT-LM (EDT_LM/edt_sim.py:175-256 -> EDT_LM/train/crossover.py:240-315: rank
selection + elitism, per child lerp(0.5) of the bases, SGD merge with the first parent's outer
momentum, uniform DNA crossover) and EDT-RL (EDT_RL/edt.py:264-299 -> EDT_RL/crossover.py:
173-201: roulette selection, per-key SLERP, reward-DNA crossover), with the CPU oracle doing the
arithmetic. The resident population must give the same members, momenta and genomes:
  * CPU, world 1 and gloo world 2 (two members per rank), oracle kernels: bit-exact;
  * MI355X, HIP kernels: EDT-LM bit-exact; SLERP within the SLERP parity bar.
The inner loop is synthetic (trained = base + seeded noise) and fitness is seeded, so the
selections do not depend on the arithmetic.
"""
import os
import random
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

SHAPES = [(33, 7), (5,), (300,), (1,), (64, 9)]
POP = 4
GENS = 3
SEG_T = [0.5, 0.43333, 0.56667, 0.5, 1.0]


def _init(m, n, dtype):
    g = torch.Generator().manual_seed(500 + m)
    return (torch.randn(n, generator=g) * 0.02).to(dtype)


def _noise(gen, m, n):
    g = torch.Generator().manual_seed(10_000 * gen + m)
    return torch.randn(n, generator=g) * 1e-3


def _fitness(gen):
    r = random.Random(77 + gen)
    return [round(r.uniform(0, 10), 3) for _ in range(POP)]


def _genomes(kind):
    if kind == "sgd":
        return [{"dna": [m, 10 + m, 20 + m]} for m in range(POP)]
    return [{"env": {"env_name": "arena", "reward_dna": [m, m + 1, m + 2, m + 3, m + 4, m + 5], "agents": []}}
            for m in range(POP)]


def _dtype(kind):
    return torch.bfloat16 if kind == "sgd" else torch.float32


def _scale(gen):
    from evolutionarydistributedtraining_amd.schedule import roulette_scale
    return roulette_scale(gen + 1, 10)


def run_resident(kind, device, kernels=None, comm=None, exchange="per_child", exchange_groups=1):
    """The resident population over GENS generations; returns this rank's members. comm: a
    collectives.Collectives (virtual ranks); the host RNGs are seeded by rank 0 only (they are
    process-global, and only rank 0 draws)."""
    from evolutionarydistributedtraining_amd.params import ParamLayout
    from evolutionarydistributedtraining_amd.population import ResidentPopulation
    layout = ParamLayout(SHAPES)
    n, dt = layout.total, _dtype(kind)
    if comm is None or comm.rank == 0:
        random.seed(7)
        np.random.seed(7)
    pop = ResidentPopulation(layout, dt, device, _genomes(kind), kind=kind, elitism=1 if kind == "sgd" else 0,
                             seg_t=SEG_T if kind == "slerp" else None, kernels=kernels, comm=comm,
                             exchange=exchange, exchange_groups=exchange_groups)
    for m in pop.local_members():
        (pop.base(m) if kind == "sgd" else pop.params(m)).copy_(_init(m, n, dt))
    for gen in range(GENS):
        pop.begin_inner()
        for m in pop.local_members():
            t = pop.trained(m) if kind == "sgd" else pop.params(m)
            t.copy_((t.cpu().float() + _noise(gen, m, n)).to(dt))
        if kind == "sgd":
            pop.step(_fitness(gen))
        else:   # the RL master samples each child's opponents right after its crossover
            pool = [f"member{m}/Gen{gen + 1:04d}/Policy" for m in range(POP)]
            pop.step(_fitness(gen), scale=_scale(gen),
                     child_hook=lambda c, g: g["env"].__setitem__("agents", random.sample(pool, 2)))
    out = {}
    for m in pop.local_members():
        if kind == "sgd":
            out[m] = {"base": pop.base(m).cpu(), "mom": pop.outer_momentum(m).cpu()}
        else:
            out[m] = {"params": pop.params(m).cpu()}
    return out, pop.genomes


def reference_flow(kind, oracle):
    """The reference's generation loop restated with the oracle's arithmetic."""
    from evolutionarydistributedtraining_amd import schedule
    from evolutionarydistributedtraining_amd.merge import uniform_dna_crossover
    from evolutionarydistributedtraining_amd.params import ParamLayout
    layout = ParamLayout(SHAPES)
    n, dt, offs = layout.total, _dtype(kind), layout.offsets
    random.seed(7)
    np.random.seed(7)
    genomes = _genomes(kind)
    base = [_init(m, n, dt) for m in range(POP)]
    mom = [None] * POP                      # outer_optim.pt of each member's GenN dir
    for gen in range(GENS):
        if kind == "sgd":
            trained = [(b.float() + _noise(gen, m, n)).to(dt) for m, b in enumerate(base)]
        else:
            base = [(b.float() + _noise(gen, m, n)).to(dt) for m, b in enumerate(base)]
        fit = _fitness(gen)
        all_g = []
        for m, g in enumerate(genomes):
            g = dict(g)
            g.update(fitness=fit[m], model_path=f"member{m}/Gen{gen:04d}")
            all_g.append(g)
        if kind == "sgd":
            sel = schedule.rank_based_selection(all_g, POP - 1)
            sel += [(e, e) for e in sorted(all_g, key=lambda g: g["fitness"], reverse=True)[:1]]
        else:
            sel = schedule.roulette_wheel_selection(all_g, POP, _scale(gen))
        idx = {g["model_path"]: m for m, g in enumerate(all_g)}
        new_base, new_mom, new_genomes = [], [], []
        for c, (g1, g2) in enumerate(sel):
            i, j = idx[g1["model_path"]], idx[g2["model_path"]]
            p1, p2 = dict(g1), dict(g2)
            for p in (p1, p2):
                p.pop("p1", None)
                p.pop("p2", None)
            if kind == "sgd":
                donor = mom[i] if mom[i] is not None else mom[j]
                if donor is None and gen > 0:
                    raise NotImplementedError
                m_out = donor.clone() if donor is not None else torch.zeros(n, dtype=dt)
                out = torch.empty(n, dtype=dt)
                oracle.pair_merge(base[i], base[j], trained[i], trained[j], out, m_out, donor is not None,
                                  0.7, 0.9, True)
                new_mom.append(m_out)
                new_genomes.append({"fitness": 0.0, "model_path": f"member{c}/Gen{gen + 1:04d}",
                                    "dna": uniform_dna_crossover(p1["dna"], p2["dna"]), "p1": p1, "p2": p2})
            else:
                out = torch.cat([oracle.slerp(SEG_T[s], base[i][offs[s]:offs[s + 1]], base[j][offs[s]:offs[s + 1]])
                                 for s in range(len(SHAPES))]).to(dt)
                env = p1["env"]
                new_genomes.append({"model_path": f"member{c}/Gen{gen + 1:04d}",
                                    "env": {"env_name": env["env_name"],
                                            "reward_dna": uniform_dna_crossover(env["reward_dna"],
                                                                                p2["env"]["reward_dna"]),
                                            "agents": []},
                                    "p1": p1, "p2": p2})
                # EDT_RL/edt.py:290-294: opponents sampled right after each crossover()
                pool = [f"member{m}/Gen{gen + 1:04d}/Policy" for m in range(POP)]
                new_genomes[-1]["env"]["agents"] = random.sample(pool, 2)
            new_base.append(out)
        base, genomes = new_base, new_genomes
        if kind == "sgd":
            mom = new_mom
    return base, mom, genomes


def _bits(t):
    return t.view(torch.int16) if t.dtype == torch.bfloat16 else t.view(torch.int32)


@pytest.mark.parametrize("kind", ["sgd", "slerp"])
def test_resident_world1_matches_reference_flow(oracle, kind):
    from tests.oracle_kernels import OracleKernels
    got, genomes = run_resident(kind, "cpu", OracleKernels(oracle))
    base, mom, want_genomes = reference_flow(kind, oracle)
    assert genomes == want_genomes
    for m in range(POP):
        if kind == "sgd":
            assert torch.equal(_bits(got[m]["base"]), _bits(base[m])), m
            assert torch.equal(_bits(got[m]["mom"]), _bits(mom[m])), m
        else:
            assert torch.equal(_bits(got[m]["params"]), _bits(base[m])), m


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _world_worker(rank, world, port, kind, outdir):
    import torch.distributed as dist

    from oracle import oracle
    from tests.oracle_kernels import OracleKernels
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    got, genomes = run_resident(kind, "cpu", OracleKernels(oracle))
    torch.save({"members": got, "genomes": genomes}, os.path.join(outdir, f"r{rank}.pt"))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.slow
@pytest.mark.parametrize("kind", ["sgd", "slerp"])
def test_resident_world2_matches_world1(tmp_path, oracle, kind):
    world = 2
    mp.start_processes(_world_worker, args=(world, _free_port(), kind, str(tmp_path)), nprocs=world,
                       join=True, start_method="spawn")
    res = [torch.load(tmp_path / f"r{r}.pt", weights_only=True) for r in range(world)]
    base, mom, want_genomes = reference_flow(kind, oracle)
    for r in range(world):
        assert res[r]["genomes"] == want_genomes
        assert sorted(res[r]["members"]) == [2 * r, 2 * r + 1]
        for m, d in res[r]["members"].items():
            if kind == "sgd":
                assert torch.equal(_bits(d["base"]), _bits(base[m])), m
                assert torch.equal(_bits(d["mom"]), _bits(mom[m])), m
            else:
                assert torch.equal(_bits(d["params"]), _bits(base[m])), m


def _check_world(res, world, kind, oracle, slerp_tol=None):
    base, mom, want_genomes = reference_flow(kind, oracle)
    per = POP // world
    for r in range(world):
        got, genomes = res[r]
        assert genomes == want_genomes
        assert sorted(got) == list(range(r * per, (r + 1) * per))
        for m, d in got.items():
            if kind == "sgd":
                assert torch.equal(_bits(d["base"]), _bits(base[m])), m
                assert torch.equal(_bits(d["mom"]), _bits(mom[m])), m
            elif slerp_tol is None:
                assert torch.equal(_bits(d["params"]), _bits(base[m])), m
            else:
                diff = (d["params"] - base[m]).abs()
                assert (diff <= slerp_tol * base[m].abs() + 1e-8).all(), (m, diff.max().item())


@pytest.mark.parametrize("world", [2, 4])
@pytest.mark.parametrize("kind", ["sgd", "slerp"])
def test_resident_virtual_ranks_match_reference_flow(oracle, kind, world):
    """The same generations on `world` virtual ranks (collectives.VirtualWorld, one process):
    members spread P / world per rank, parents exchanged by the grouped p2p, genomes broadcast."""
    from evolutionarydistributedtraining_amd.collectives import VirtualWorld
    from tests.oracle_kernels import OracleKernels
    res = VirtualWorld(world).run(lambda comm: run_resident(kind, "cpu", OracleKernels(oracle), comm=comm))
    _check_world(res, world, kind, oracle)


def test_resident_sharded_exchange_virtual_ranks(oracle):
    """exchange="sharded" (one member per rank, link-balanced) on 4 virtual ranks, EDT-LM: the
    same members, momenta and genomes as the reference flow, bit for bit."""
    from evolutionarydistributedtraining_amd.collectives import VirtualWorld
    from tests.oracle_kernels import ChunkGramKernels
    res = VirtualWorld(POP).run(lambda comm: run_resident("sgd", "cpu", ChunkGramKernels(oracle), comm=comm,
                                                          exchange="sharded"))
    _check_world(res, POP, "sgd", oracle)


@pytest.mark.gpu
@pytest.mark.parametrize("kind,groups", [("sgd", 1), ("slerp", 1), ("slerp", 3)])
def test_resident_gpu_sharded_exchange(oracle, kind, groups):
    """exchange="sharded" with the HIP kernels on 4 virtual ranks: EDT-LM bit-exact, SLERP within
    the SLERP bar of the reference flow (also with the exchanges pipelined over 3 chunk groups)."""
    from evolutionarydistributedtraining_amd.collectives import VirtualWorld
    dev = torch.device("cuda:0")
    res = VirtualWorld(POP).run(lambda comm: run_resident(kind, dev, comm=comm, exchange="sharded",
                                                          exchange_groups=groups))
    _check_world(res, POP, kind, oracle, slerp_tol=1e-5)


@pytest.mark.gpu
@pytest.mark.parametrize("world", [2, 4])
@pytest.mark.parametrize("kind", ["sgd", "slerp"])
def test_resident_gpu_virtual_ranks(oracle, kind, world):
    """The HIP kernels inside the N-rank generation schedule on one MI355X (virtual ranks):
    EDT-LM bit-exact, SLERP within the SLERP parity bar."""
    from evolutionarydistributedtraining_amd.collectives import VirtualWorld
    dev = torch.device("cuda:0")
    res = VirtualWorld(world).run(lambda comm: run_resident(kind, dev, comm=comm))
    _check_world(res, world, kind, oracle, slerp_tol=1e-5)


def test_resident_rejects_missing_momentum(oracle):
    """Past generation 0 a child whose parents have no outer state is an error, as in
    EDT_LM/train/crossover.py:226-227."""
    from evolutionarydistributedtraining_amd.params import ParamLayout
    from evolutionarydistributedtraining_amd.population import ResidentPopulation
    from tests.oracle_kernels import OracleKernels
    pop = ResidentPopulation(ParamLayout(SHAPES), torch.bfloat16, "cpu", _genomes("sgd"),
                             kernels=OracleKernels(oracle))
    pop.generation = 1
    with pytest.raises(NotImplementedError):
        pop.crossover([(0, 1), (1, 2), (2, 3), (3, 0)])


@pytest.mark.gpu
@pytest.mark.parametrize("kind", ["sgd", "slerp"])
def test_resident_gpu_matches_reference_flow(oracle, kind):
    got, genomes = run_resident(kind, torch.device("cuda:0"))
    base, mom, want_genomes = reference_flow(kind, oracle)
    assert genomes == want_genomes
    for m in range(POP):
        if kind == "sgd":
            assert torch.equal(_bits(got[m]["base"]), _bits(base[m])), m
            assert torch.equal(_bits(got[m]["mom"]), _bits(mom[m])), m
        else:
            # SLERP parity bar: the fp64 dot vs the reference's fp32 one
            diff = (got[m]["params"] - base[m]).abs()
            assert (diff <= 1e-5 * base[m].abs() + 1e-8).all(), (m, diff.max().item())


def test_resident_save_load_resumes_exactly(tmp_path, oracle):
    """Three generations straight vs two, save(), a fresh population load()ed, one more: the
    same members, momenta and genomes (host RNG states restored with them)."""
    from evolutionarydistributedtraining_amd.params import ParamLayout
    from evolutionarydistributedtraining_amd.population import ResidentPopulation
    from tests.oracle_kernels import OracleKernels
    layout = ParamLayout(SHAPES)
    n, dt = layout.total, torch.bfloat16

    def fresh():
        return ResidentPopulation(layout, dt, "cpu", _genomes("sgd"), elitism=1, kernels=OracleKernels(oracle))

    def gens(pop, lo, hi):
        for gen in range(lo, hi):
            pop.begin_inner()
            for m in pop.local_members():
                t = pop.trained(m)
                t.copy_((t.float() + _noise(gen, m, n)).to(dt))
            pop.step(_fitness(gen))

    random.seed(7)
    np.random.seed(7)
    a = fresh()
    for m in a.local_members():
        a.base(m).copy_(_init(m, n, dt))
    gens(a, 0, GENS)
    random.seed(7)
    np.random.seed(7)
    b = fresh()
    for m in b.local_members():
        b.base(m).copy_(_init(m, n, dt))
    gens(b, 0, GENS - 1)
    b.save(str(tmp_path / "ckpt"))
    random.seed(12345)                      # disturb the host RNGs: load() must restore them
    np.random.seed(12345)
    c = fresh()
    c.load(str(tmp_path / "ckpt"))
    assert c.generation == GENS - 1
    gens(c, GENS - 1, GENS)
    assert c.genomes == a.genomes
    for m in range(POP):
        assert torch.equal(_bits(c.base(m)), _bits(a.base(m))), m
        assert torch.equal(_bits(c.outer_momentum(m)), _bits(a.outer_momentum(m))), m


def edt_master_flow(oracle):
    """EDT_LM/edt.py's generation loop restated (the distributed master): tournament selection
    over this generation and the previous one (:213-247), elites from this one, the worker's
    crossover.py per child; the previous generation's base / trained / outer_optim.pt stay
    addressable (its GenN-1 dirs)."""
    from evolutionarydistributedtraining_amd import schedule
    from evolutionarydistributedtraining_amd.merge import uniform_dna_crossover
    from evolutionarydistributedtraining_amd.params import ParamLayout
    layout = ParamLayout(SHAPES)
    n, dt = layout.total, torch.bfloat16
    random.seed(11)
    np.random.seed(11)
    genomes = _genomes("sgd")
    base = [_init(m, n, dt) for m in range(POP)]
    mom = [None] * POP
    prev = None                                  # (genomes with fitness, base, trained, mom)
    for gen in range(GENS + 1):
        trained = [(b.float() + _noise(gen, m, n)).to(dt) for m, b in enumerate(base)]
        fit = _fitness(gen)
        cur = []
        for m, g in enumerate(genomes):
            g = dict(g)
            g.update(fitness=fit[m], model_path=f"member{m}/Gen{gen:04d}")
            cur.append(g)
        pool = cur + (prev[0] if prev else [])
        sel = schedule.tournament_selection(pool, POP - 1)
        sel += [(e, e) for e in sorted(cur, key=lambda g: g["fitness"], reverse=True)[:1]]
        idx = {g["model_path"]: q for q, g in enumerate(pool)}
        all_b = base + (prev[1] if prev else [])
        all_t = trained + (prev[2] if prev else [])
        all_m = mom + (prev[3] if prev else [])
        new_b, new_m, new_g = [], [], []
        for c, (g1, g2) in enumerate(sel):
            i, j = idx[g1["model_path"]], idx[g2["model_path"]]
            p1, p2 = dict(g1), dict(g2)
            for p in (p1, p2):
                p.pop("p1", None)
                p.pop("p2", None)
            donor = all_m[i] if all_m[i] is not None else all_m[j]
            m_out = donor.clone() if donor is not None else torch.zeros(n, dtype=dt)
            out = torch.empty(n, dtype=dt)
            oracle.pair_merge(all_b[i], all_b[j], all_t[i], all_t[j], out, m_out, donor is not None, 0.7, 0.9, True)
            new_b.append(out)
            new_m.append(m_out)
            new_g.append({"fitness": 0.0, "model_path": f"member{c}/Gen{gen + 1:04d}",
                          "dna": uniform_dna_crossover(p1["dna"], p2["dna"]), "p1": p1, "p2": p2})
        prev = (cur, base, trained, mom)
        base, mom, genomes = new_b, new_m, new_g
    return base, mom, genomes


def run_edt_master(device, kernels=None):
    from evolutionarydistributedtraining_amd.params import ParamLayout
    from evolutionarydistributedtraining_amd.population import ResidentPopulation
    layout = ParamLayout(SHAPES)
    n, dt = layout.total, torch.bfloat16
    random.seed(11)
    np.random.seed(11)
    pop = ResidentPopulation(layout, dt, device, _genomes("sgd"), elitism=1, keep_previous=True, kernels=kernels)
    for m in pop.local_members():
        pop.base(m).copy_(_init(m, n, dt))
    used = []
    for gen in range(GENS + 1):
        pop.begin_inner()
        for m in pop.local_members():
            t = pop.trained(m)
            t.copy_((t.cpu().float() + _noise(gen, m, n)).to(dt))
        used += pop.step(_fitness(gen), method="tournament_pool")
    return {m: (pop.base(m).cpu(), pop.outer_momentum(m).cpu()) for m in pop.local_members()}, pop.genomes, used


def test_edt_master_tournament_pool_world1(oracle):
    from tests.oracle_kernels import OracleKernels
    got, genomes, used = run_edt_master("cpu", OracleKernels(oracle))
    base, mom, want = edt_master_flow(oracle)
    assert genomes == want
    assert any(max(p) >= POP for p in used)       # previous-generation parents were drawn
    for m in range(POP):
        assert torch.equal(_bits(got[m][0]), _bits(base[m])), m
        assert torch.equal(_bits(got[m][1]), _bits(mom[m])), m


def _edt_master_worker(rank, world, port, outdir):
    import torch.distributed as dist

    from oracle import oracle
    from tests.oracle_kernels import OracleKernels
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    got, genomes, _ = run_edt_master("cpu", OracleKernels(oracle))
    torch.save({"members": got, "genomes": genomes}, os.path.join(outdir, f"m{rank}.pt"))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.slow
def test_edt_master_tournament_pool_world2(tmp_path, oracle):
    """Previous-generation parents live on their own ranks: the exchange ships them too."""
    world = 2
    mp.start_processes(_edt_master_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True,
                       start_method="spawn")
    base, mom, want = edt_master_flow(oracle)
    for r in range(world):
        res = torch.load(tmp_path / f"m{r}.pt", weights_only=True)
        assert res["genomes"] == want
        for m, (b, mo) in res["members"].items():
            assert torch.equal(_bits(b), _bits(base[m])), m
            assert torch.equal(_bits(mo), _bits(mom[m])), m


@pytest.mark.gpu
def test_edt_master_tournament_pool_gpu(oracle):
    got, genomes, used = run_edt_master(torch.device("cuda:0"))
    base, mom, want = edt_master_flow(oracle)
    assert genomes == want
    for m in range(POP):
        assert torch.equal(_bits(got[m][0]), _bits(base[m])), m
        assert torch.equal(_bits(got[m][1]), _bits(mom[m])), m


def test_evomerge_master_genomes(oracle):
    """EDT_EVOMERGE/edt.py: rank selection + elitism, SLERP children of DNA genomes (the
    EVOMERGE worker writes the EDT-LM genome record, EDT_EVOMERGE/train/crossover.py:214-227)."""
    from evolutionarydistributedtraining_amd.params import ParamLayout
    from evolutionarydistributedtraining_amd.population import ResidentPopulation
    from tests.oracle_kernels import OracleKernels
    random.seed(3)
    np.random.seed(3)
    pop = ResidentPopulation(ParamLayout(SHAPES), torch.float32, "cpu", _genomes("sgd"), kind="slerp",
                             seg_t=SEG_T, elitism=1, kernels=OracleKernels(oracle))
    for m in pop.local_members():
        pop.params(m).copy_(_init(m, ParamLayout(SHAPES).total, torch.float32))
    pairs = pop.step(_fitness(0), method="rank")
    assert len(pairs) == POP and pairs[-1][0] == pairs[-1][1]          # the elite self-pair
    for c, g in enumerate(pop.genomes):
        assert set(g) == {"fitness", "model_path", "dna", "p1", "p2"} and g["fitness"] == 0.0
        assert g["model_path"] == f"member{c}/Gen0001"
