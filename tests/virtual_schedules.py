"""Shared drivers for the multi-rank schedules run as N virtual ranks in one process
(collectives.VirtualWorld): the CPU tests run them with the oracle as the kernels, the GPU tests
with the HIP kernels on one MI355X. Each returns what every rank holds after the schedule, with
the sharded momentum reassembled in parameter order."""
from __future__ import annotations

import torch

from evolutionarydistributedtraining_amd.collectives import VirtualWorld
from evolutionarydistributedtraining_amd.params import ParamLayout


def population(shapes, tdt, wdt, k_total, steps, seed=99, device="cpu"):
    """theta ~ N(0, .02^2) and `steps` generations of k_total workers = theta + N(0, (s+1) 1e-3)."""
    layout = ParamLayout(shapes)
    g = torch.Generator().manual_seed(seed)
    theta = (torch.randn(layout.total, generator=g) * 0.02).to(tdt)
    gens = []
    for s in range(steps):
        gens.append([(theta.float() + torch.randn(layout.total, generator=g) * 1e-3 * (s + 1)).to(wdt).to(device)
                     for _ in range(k_total)])
    return layout, theta.to(device), gens


def run_sharded(world, layout, tdt, wdt, theta0, gens, device, kernels=None, mode="exact", broadcast="theta",
                bucket_elems=1024, lr=0.7, mu=0.9, nesterov=True):
    """ShardedOuterSync on `world` virtual ranks (K_local = len(gens[0]) / world). Returns per rank
    {"theta" (gather_theta), "mom" (rank 0: the momentum reassembled), "workers", "sync"}."""
    from evolutionarydistributedtraining_amd.distributed import ShardedOuterSync
    k_total = len(gens[0])
    k_local = k_total // world
    vw = VirtualWorld(world)

    def body(comm):
        sync = ShardedOuterSync(layout, tdt, wdt, k_local, device, lr, mu, nesterov, mode=mode,
                                bucket_elems=bucket_elems, kernels=kernels, broadcast=broadcast, comm=comm)
        sync.theta.flat.copy_(theta0)
        for workers in gens:
            for j, arena in enumerate(sync.workers):
                arena.flat.copy_(workers[comm.rank * k_local + j])
            sync.step()
        left = [w.flat.clone() for w in sync.workers]        # what the step left (broadcast="workers")
        theta = sync.gather_theta().clone()
        shards = comm.all_gather_object(None if sync.mom_shard is None else sync.mom_shard.clone())
        return {"theta": theta, "mom_shards": shards, "workers": left, "buckets": sync.buckets,
                "mode": sync.mode, "broadcast": sync.broadcast, "n_pad": sync.n_pad}

    res = vw.run(body)
    r0 = res[0]
    mom = None
    if r0["mom_shards"][0] is not None:
        mom = torch.empty(r0["n_pad"], dtype=tdt, device=theta0.device)
        off = [0] * world
        for b, e in r0["buckets"]:
            per = (e - b) // world
            for r in range(world):
                mom[b + r * per:b + (r + 1) * per] = r0["mom_shards"][r][off[r]:off[r] + per]
                off[r] += per
        mom = mom[:layout.total]
    for r in res:
        r["mom"] = mom
    return res


def ulp(x, dt):
    a = x.float().abs().clamp_min(torch.finfo(dt).tiny)
    return torch.exp2(torch.floor(torch.log2(a)) - (23 if dt == torch.float32 else 7))


def reduce_tol(th_ref, mom_ref, tdt, lr=0.7, gens=None, mu=0.9):
    """The reduce schedule's bound against the reference's sequential worker order:
    2 ulp(theta) + 4 ulp(|update| + lr(|buf'| + mu|buf|)), plus — given the workers — the
    reassociation of the K-term mean: the reference accumulates it in theta's dtype (unit
    roundoff u: 2^-24 fp32, 2^-8 bf16), the schedule in fp32 across ranks, so the two sums differ
    by at most 2 K u sum_k |delta_k / K|; that reaches theta through lr (1 + mu) (Nesterov),
    counted twice per step for the carry into the next step's deltas."""
    scale = lr * (mom_ref.float().abs() * 1.9)
    tol = 2 * ulp(th_ref, tdt) + 4 * ulp(scale, tdt)
    if gens is not None:
        u = 2.0 ** -24 if tdt == torch.float32 else 2.0 ** -8
        for ws in gens:
            K = len(ws)
            s = sum((w.float() - th_ref.float()).abs() for w in ws) / K
            tol = tol + 2 * K * u * lr * (1 + mu) * s * 2
    return tol


def reduce_reference(oracle, theta, gens, world, lr=0.7, mu=0.9, nesterov=True):
    """The reduce schedule's exact result when the cross-rank sum runs in rank order (what the
    virtual ranks do; RCCL's order is its own): per rank the fp32 partial of its local workers
    (oracle.delta_partial), partials summed rank 0..N-1, then the SGD step (oracle.sgd_apply)."""
    th = theta.clone()
    mom = torch.zeros_like(th)
    for i, ws in enumerate(gens):
        K = len(ws)
        kl = K // world
        total = None
        for r in range(world):
            acc = torch.zeros(th.numel(), dtype=torch.float32, device=th.device)
            oracle.delta_partial(th, ws[r * kl:(r + 1) * kl], K, acc, False)
            total = acc if total is None else total.add_(acc)
        oracle.sgd_apply(th, total, mom, i > 0, lr, mu, nesterov)
    return th, mom


def bits(t):
    return t.view(torch.int32) if t.dtype == torch.float32 else t.view(torch.int16)
