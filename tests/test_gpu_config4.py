"""BASELINE configs[4] at its named shape: "EDT_RL/crossover.py path: population-of-8 weighted-blend
crossover on 7B-param tensors". Eight Qwen2.5-7B bodies (7.07B bf16 parameters, 338 tensors) are
SLERP-crossed into eight children (EDT_RL/edt.py:286-299 -> EDT_RL/crossover.py:84-135 per child;
EVOMERGE's bf16 form, EDT_EVOMERGE/train/crossover.py:104-146).

  * world 1, the whole population resident on one MI355X (8 members + 8 children = 226 GB of the
    288 GB) through ResidentPopulation(kind="slerp"), three generations so that every population
    kernel form runs: lineage members (the speculative single pass, every segment in the lerp
    branch), independent members (the speculative pass + its SLERP-branch redo), and their
    children (the Gram stats pass + member-major blends, chosen from the previous dots). Every child
    is bit-identical to edt_slerp_merge (two-pass) on its two parents, and sampled small segments
    are within the golden bar of the oracle (numpy restatement of the reference).
  * the link-balanced ShardedPopulationCrossover at world 4 (virtual ranks, one member per rank)
    on the same 7B body: every child bit-identical to edt_slerp_merge.

EDT_RECORD_DIR=<dir> writes the per-generation times to <dir>/config4_times.json."""
from __future__ import annotations

import json
import os
import time

import pytest
import torch

pytestmark = pytest.mark.gpu

BF = torch.bfloat16


@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.skip("needs a HIP device")
    return torch.device("cuda:0")


def _record(key, value):
    d = os.environ.get("EDT_RECORD_DIR")
    if not d:
        return
    os.makedirs(d, exist_ok=True)
    path = os.path.join(d, "config4_times.json")
    data = {}
    if os.path.exists(path):
        with open(path) as f:
            data = json.load(f)
    data[key] = value
    with open(path, "w") as f:
        json.dump(data, f, indent=1)


def _fill(dst, gen, scale, base=None, rel=0.0):
    """dst = N(0, scale) (base is None) or base + N(0, rel * scale), in 256 Mi-element pieces."""
    step = 1 << 28
    for s in range(0, dst.numel(), step):
        e = min(dst.numel(), s + step)
        x = torch.randn(e - s, device=dst.device, generator=gen) * scale
        if base is not None:
            x = base[s:e].float() + x * rel
        dst[s:e] = x.to(dst.dtype)


def _free_hbm(dev):
    """Bytes the device can still allocate: everything this process's caching allocator holds from
    earlier tests is released first."""
    import gc
    gc.collect()
    torch.cuda.synchronize(dev)
    torch.cuda.empty_cache()
    free, _ = torch.cuda.mem_get_info(dev)
    return free


def _small_segments(lay, count=12):
    return [s for s in range(len(lay)) if lay.numels[s] <= 200_000][:count]


def _check_children(oracle, lay, plan, parents, pairs, children, t, want):
    """Every child bit-identical to edt_slerp_merge (two-pass) on its parents; sampled small
    segments within the golden bar of the oracle (bf16 output: the oracle's fp32 result within the
    coefficient gap of the two dots plus two bf16 ulps, as test_gpu_fullsize)."""
    from evolutionarydistributedtraining_amd import ops
    small = _small_segments(lay)
    th = t.cpu()
    for c, (i, j) in enumerate(pairs):
        ops.slerp_arena(plan, parents[i], parents[j], want, t, speculate=False)
        torch.cuda.synchronize()
        assert torch.equal(children[c].view(torch.int16), want.view(torch.int16)), f"child {c} of {(i, j)}"
        if c >= 2:
            continue
        coef = plan.coef[:len(lay)].cpu()
        for s in small:
            a, b = lay.offsets[s], lay.offsets[s + 1]
            x, y = parents[i][a:b].cpu(), parents[j][a:b].cpu()
            res, _, _ = oracle.slerp_parts(float(th[s]), x, y)
            rc0, rc1, _ = oracle.slerp_coefficients(float(th[s]), x, y)
            ref = torch.from_numpy(res).bfloat16().float()
            c0, c1 = coef[s].tolist()
            tol = 1.01 * (abs(c0 - float(rc0)) * x.float().abs() + abs(c1 - float(rc1)) * y.float().abs())
            tol = tol + 2e-6 * (abs(c0) * x.float().abs() + abs(c1) * y.float().abs())
            tol = tol + 2 * torch.exp2(torch.floor(torch.log2(ref.abs().clamp_min(1e-38))) - 7)
            got = children[c][a:b].cpu().float()
            assert ((got - ref).abs() <= tol).all(), (c, lay.names[s])


def test_config4_resident_population_8x7b(oracle, dev):
    from evolutionarydistributedtraining_amd import ops
    from evolutionarydistributedtraining_amd.layouts import qwen2p5_7b_body
    from evolutionarydistributedtraining_amd.population import ResidentPopulation
    lay = qwen2p5_7b_body()
    P, N = lay.total, 8
    free = _free_hbm(dev)
    need = (2 * N + 1) * P * 2
    if free < need + (4 << 30):
        pytest.skip(f"needs {need / 1e9:.0f} GB of HBM, {free / 1e9:.0f} GB free")
    gen = torch.Generator(device=dev).manual_seed(4)
    genomes = [{"env": {"env_name": "ivy", "reward_dna": [m % 3, 1, 0], "agents": []}} for m in range(N)]
    t = torch.rand(len(lay), dtype=torch.float64, generator=torch.Generator().manual_seed(4)).tolist()
    pop = ResidentPopulation(lay, BF, dev, genomes, kind="slerp", seg_t=t)
    tdev = pop._t
    # generation 0: members of one lineage (one base + 0.5 % per member): every segment in the
    # lerp branch, the speculative single pass
    base = torch.empty(P, dtype=BF, device=dev)
    _fill(base, gen, 0.02)
    for m in range(N):
        _fill(pop.params(m), gen, 0.02, base=base, rel=0.005)
    del base
    want = torch.empty(P, dtype=BF, device=dev)
    pair_sets = [[((3 * c + 1) % N, (5 * c + 2) % N) for c in range(N)],
                 [((c + 1) % N, (c + 3) % N) for c in range(N)],
                 [((2 * c) % N, (2 * c + 5) % N) for c in range(N)]]
    times = {}
    for g, pairs in enumerate(pair_sets):
        if g == 1:       # independent members: the speculative pass redoes every segment
            for m in range(N):
                _fill(pop.params(m), gen, 0.02)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        pop.crossover(pairs)
        torch.cuda.synchronize()
        times[f"gen{g}_ms"] = round(1e3 * (time.perf_counter() - t0), 2)
        dots = pop._plan._pop_dots.cpu()
        if g == 0:
            assert bool((dots.abs() > 0.9995).all()), "lineage members must all take the lerp branch"
        else:
            assert bool((dots.abs() <= 0.9995).float().mean() > 0.9), "independent members: the SLERP branch"
        # the parents are the arenas swapped out by the crossover
        parents = pop._child
        _check_children(oracle, lay, pop._plan, parents, pairs, pop._params, tdev, want)
    times["forms"] = ["speculative, lerp branch", "speculative + redo", "gram + member-major blend"]
    _record("resident_8x7b", times)


def test_config4_sharded_world4_7b(dev):
    from evolutionarydistributedtraining_amd import ops
    from evolutionarydistributedtraining_amd.collectives import VirtualWorld
    from evolutionarydistributedtraining_amd.distributed import ShardedPopulationCrossover
    from evolutionarydistributedtraining_amd.layouts import qwen2p5_7b_body
    lay = qwen2p5_7b_body()
    P, N = lay.total, 4
    free = _free_hbm(dev)
    need = (4 * N + 1) * P * 2
    if free < need + (4 << 30):
        pytest.skip(f"needs {need / 1e9:.0f} GB of HBM, {free / 1e9:.0f} GB free")
    gen = torch.Generator(device=dev).manual_seed(44)
    members = []
    base = torch.empty(P, dtype=BF, device=dev)
    _fill(base, gen, 0.02)
    for m in range(N):
        x = torch.empty(P, dtype=BF, device=dev)
        _fill(x, gen, 0.02, base=base, rel=0.005 if m % 2 else 0.05)
        members.append(x)
    del base
    pairs = [(1, 2), (3, 0), (2, 2), (0, 3)]
    t = torch.rand(len(lay), dtype=torch.float64, device=dev, generator=gen)

    def body(comm):
        sp = ShardedPopulationCrossover(lay, BF, dev, comm=comm)
        out = torch.empty(P, dtype=BF, device=dev)
        sp.slerp_step(members[comm.rank], pairs, t, out)
        torch.cuda.synchronize()
        del sp
        return out

    t0 = time.perf_counter()
    res = VirtualWorld(N, timeout=900).run(body)
    _record("sharded_world4_7b_s", round(time.perf_counter() - t0, 2))
    plan = ops.make_slerp_plan(lay.offsets, dev)
    want = torch.empty(P, dtype=BF, device=dev)
    for c, (i, j) in enumerate(pairs):
        ops.slerp_arena(plan, members[i], members[j], want, t, speculate=False)
        torch.cuda.synchronize()
        assert torch.equal(res[c].view(torch.int16), want.view(torch.int16)), c
