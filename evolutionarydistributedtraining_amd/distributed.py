"""DiLoCo outer step across GPUs: one process per GPU, RCCL over xGMI (torch.distributed "nccl").

The reference has no collectives: its "gather" is K x `from_pretrained` of the workers'
checkpoints on a shared disk and its "broadcast" is K x `save_pretrained` (EDT_LM/diloco.py:
231-235, 302-308). Here the population is resident in HBM across the node and the cross-replica
mean is a real exchange step. Two schedules, both bucketed so RCCL traffic on the comm stream
overlaps the HBM-bound kernels on the compute stream:

  mode="reduce"  each rank fuses its local workers into an fp32 partial sum (edt_delta_partial),
                 reduce-scatter(sum, fp32) -> SGD on the owned shard (momentum sharded 1/N,
                 edt_sgd_apply) -> all-gather of theta. Wire bytes per rank and step:
                 (N-1)/N * P * (4 + b_g). Summation order across ranks differs from the
                 reference's sequential order: fp32 <= 2 ulp, bf16 <= 1 bf16 ulp.
  mode="exact"   all-to-all of the raw worker shards to their owners, then the single-GPU fused
                 kernel on each shard (the reference's worker order, bit-exact), all-gather of
                 theta. Wire bytes: (N-1)/N * P * (K_local * b_w + b_g).
  broadcast      what the all-gather delivers to every rank. "theta": the full master replica
                 (theta's dtype). "workers" (exact mode only): the new theta rounded to the worker
                 dtype, straight into every local worker arena — the start of the next inner
                 loop, which is all the reference ships to the workers (diloco.py:302-308 saves
                 the base to every worker dir; the bf16 workers load it rounded). The fp32 master
                 then stays sharded (each rank updates only the shard it owns; `gather_theta()`
                 assembles it on demand, e.g. for a checkpoint). Wire bytes:
                 (N-1)/N * P * (K_local + 1) * b_w.
  mode="auto" / broadcast="auto" (defaults) pick the combination with the fewest wire bytes:
  at K = 8 bf16 workers, fp32 theta: N = 2 reduce/theta (8 B/elem), N = 4 and 8 exact/workers
  (6 and 4 B/elem).

Every rank holds 1/N of the momentum and owns contiguous shards of every bucket.
"""
from __future__ import annotations

import math

import torch

from . import ops as _ops
from .collectives import Collectives, TorchCollectives
from .diloco import check_sgd_hparams
from .params import ParamArena, ParamLayout


class ShardedOuterSync:
    def __init__(self, layout: ParamLayout, theta_dtype: torch.dtype, worker_dtype: torch.dtype,
                 k_local: int, device, lr: float = 0.7, momentum: float = 0.9, nesterov: bool = True,
                 mode: str = "auto", bucket_elems: int = 1 << 26, group=None, kernels=None,
                 broadcast: str = "auto", comm: Collectives | None = None):
        if mode not in ("reduce", "exact", "auto") or broadcast not in ("theta", "workers", "auto"):
            raise ValueError((mode, broadcast))
        if mode == "reduce" and broadcast == "workers":
            raise ValueError("the reduce schedule needs the full theta replica (broadcast='theta')")
        check_sgd_hparams(lr, momentum, nesterov)
        # the communicator seam: torch.distributed (RCCL / gloo) by default, or N virtual ranks
        # on one device (collectives.VirtualWorld)
        self.comm = comm or TorchCollectives(group)
        self.world = self.comm.world
        self.rank = self.comm.rank
        wb = torch.empty(0, dtype=worker_dtype).element_size()
        gb = torch.empty(0, dtype=theta_dtype).element_size()
        cands = {("reduce", "theta"): 4 + gb, ("exact", "theta"): k_local * wb + gb,
                 ("exact", "workers"): (k_local + 1) * wb}
        cands = {key: v for key, v in cands.items()
                 if mode in ("auto", key[0]) and broadcast in ("auto", key[1])}
        # fewest wire bytes per element; ties go to the bit-exact schedule
        mode, broadcast = min(cands, key=lambda key: (cands[key], key[0] != "exact", key[1] != "workers"))
        self.kernels = kernels or _ops
        self.mode = mode
        self.broadcast = broadcast
        self.layout = layout
        self.lr, self.momentum, self.nesterov = lr, momentum, nesterov
        self.k_local = k_local
        self.k_total = k_local * self.world
        n = layout.total
        # buckets: multiples of world * 64 elements so every shard is 16-byte aligned
        unit = self.world * 64
        bucket = max(unit, bucket_elems // unit * unit)
        self.n = n
        self.n_pad = math.ceil(n / unit) * unit
        self.bucket = min(bucket, self.n_pad)
        self.buckets = [(b, min(b + self.bucket, self.n_pad)) for b in range(0, self.n_pad, self.bucket)]
        self.theta_buf = torch.zeros(self.n_pad, dtype=theta_dtype, device=device)
        self.theta = ParamArena(layout, theta_dtype, device, self.theta_buf[:n])
        self.worker_bufs = [torch.zeros(self.n_pad, dtype=worker_dtype, device=device) for _ in range(k_local)]
        self.workers = [ParamArena(layout, worker_dtype, device, w[:n]) for w in self.worker_bufs]
        shard_total = sum((e - b) // self.world for b, e in self.buckets)
        self.mom_shard = torch.zeros(shard_total, dtype=theta_dtype, device=device) if momentum else None
        self.has_momentum = False
        # RCCL (and the virtual ranks) reduce/gather in place; gloo gets separate buffers
        self.inplace = self.comm.inplace
        self.kernel_events = None      # a list: (start, end) HIP events around every local kernel
        if mode == "reduce":
            self.acc = torch.zeros(self.n_pad, dtype=torch.float32, device=device)
            self.acc_shard = None if self.inplace else torch.empty(shard_total, dtype=torch.float32, device=device)
        else:
            # recv[j][b:e] viewed [src rank][per]: local worker j of every rank, this rank's shard
            self.recv = [torch.empty(self.n_pad, dtype=worker_dtype, device=device) for _ in range(k_local)]

    # ---------------------------------------------------------------------------------------
    def _shard(self, b, e):
        per = (e - b) // self.world
        return b + self.rank * per, b + (self.rank + 1) * per

    def _launch(self, fn, *args):
        """A local kernel, bracketed by timing events on its launch stream when
        `kernel_events` is a list (bench.py: the per-rank HBM roofline at N > 1)."""
        if self.kernel_events is None:
            return fn(*args)
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        fn(*args)
        b.record()
        self.kernel_events.append((a, b))

    def kernel_bytes(self) -> int:
        """Algorithmic HBM bytes of one step's local kernels on this rank (steady state:
        momentum read + written). exact: the fused kernel over the owned shards with all K
        workers; reduce: the partial over the whole arena + the SGD over the owned shards."""
        wb = self.worker_bufs[0].element_size()
        gb = self.theta_buf.element_size()
        shard = self.n_pad // self.world
        mom = 2 * gb if self.momentum else 0
        if self.mode == "exact":
            return shard * (self.k_total * wb + 2 * gb + mom)
        return self.n_pad * (self.k_local * wb + gb + 4) + shard * (4 + 2 * gb + mom)

    def step(self) -> None:
        """One outer step; returns when the work is enqueued (stream-ordered, async)."""
        k = self.kernels
        mom_off = 0
        gathers = []
        if self.mode == "reduce":
            # phase 1: local partial sums, reduce-scatter each bucket as soon as it is ready
            works = []
            for b, e in self.buckets:
                self._launch(k.delta_partial, self.theta_buf[b:e], [w[b:e] for w in self.worker_bufs],
                             self.k_total, self.acc[b:e], False)
                works.append(self.comm.reduce_scatter(self._acc_out(b, e), self.acc[b:e], async_op=True))
            # phase 2: SGD on the owned shard, all-gather theta
            for (b, e), w in zip(self.buckets, works):
                w.wait()
                s0, s1 = self._shard(b, e)
                per = s1 - s0
                mom = None if self.mom_shard is None else self.mom_shard[mom_off:mom_off + per]
                self._launch(k.sgd_apply, self.theta_buf[s0:s1], self._acc_out(b, e), mom, self.has_momentum,
                             self.lr, self.momentum, self.nesterov)
                mom_off += per
                gathers.append(self._gather(b, e, s0, s1))
        else:
            # phase 1: every bucket's all-to-all, straight from the worker arenas (a worker's
            # bucket [b, e) is already laid out [dest rank][per]); one collective per local worker
            works = []
            for b, e in self.buckets:
                works.append([self.comm.all_to_all(self.recv[j][b:e], wb[b:e], async_op=True)
                              for j, wb in enumerate(self.worker_bufs)])
            # phase 2: as each bucket lands, the single-GPU fused step on the owned shard
            for (b, e), ws in zip(self.buckets, works):
                for w in ws:
                    w.wait()
                per = (e - b) // self.world
                rv = [r[b:e].view(self.world, per) for r in self.recv]
                # global worker k = src * K_local + j: the reference's worker order
                shards = [rv[j][src] for src in range(self.world) for j in range(self.k_local)]
                s0, s1 = self._shard(b, e)
                mom = None if self.mom_shard is None else self.mom_shard[mom_off:mom_off + per]
                # broadcast="workers": the HIP kernel also stores the new shard, rounded to the
                # worker dtype, into local worker 0's arena (its bucket has been sent) — the
                # rounding copy fused into the step
                fused = self.broadcast == "workers" and k is _ops
                self._launch(k.outer_step, self.theta_buf[s0:s1], shards, mom, self.has_momentum, self.lr,
                             self.momentum, self.nesterov, *([[self.worker_bufs[0][s0:s1]]] if fused else []))
                mom_off += per
                if self.broadcast == "workers":
                    gathers.append(self._gather_to_workers(b, e, s0, s1, rounded=fused))
                else:
                    gathers.append(self._gather(b, e, s0, s1))
        for g in gathers:
            g.wait()
        if self.broadcast == "workers":
            for w in self.worker_bufs[1:]:          # every local worker starts from the same theta
                w.copy_(self.worker_bufs[0])
        if self.momentum:
            self.has_momentum = True

    def _acc_out(self, b, e):
        """Reduce-scatter destination for bucket [b, e): this rank's slice of the acc buffer
        (in place, as RCCL allows: recv == send + rank * count); a separate slice elsewhere."""
        s0, s1 = self._shard(b, e)
        if self.inplace:
            return self.acc[s0:s1]
        off = sum((e2 - b2) // self.world for b2, e2 in self.buckets if b2 < b)
        return self.acc_shard[off:off + (s1 - s0)]

    def _gather(self, b, e, s0, s1):
        """All-gather the updated shards of bucket [b, e) into every rank's theta replica."""
        src = self.theta_buf[s0:s1] if self.inplace else self.theta_buf[s0:s1].clone()
        return self.comm.all_gather(self.theta_buf[b:e], src, async_op=True)

    def _gather_to_workers(self, b, e, s0, s1, rounded=False):
        """The new theta shard of bucket [b, e), rounded to the worker dtype (torch copy_: RNE;
        rounded=True: the kernel already stored it), all-gathered into local worker 0's arena
        (its bucket was consumed by the all-to-all)."""
        w0 = self.worker_bufs[0]
        if not rounded:
            w0[s0:s1].copy_(self.theta_buf[s0:s1])
        src = w0[s0:s1] if self.inplace else w0[s0:s1].clone()
        return self.comm.all_gather(w0[b:e], src, async_op=True)

    def gather_theta(self) -> torch.Tensor:
        """The full master theta on every rank (with broadcast="workers" it is kept sharded;
        this assembles it, e.g. for a checkpoint). Returns the flat theta (length P)."""
        if self.broadcast == "workers":
            for b, e in self.buckets:
                s0, s1 = self._shard(b, e)
                src = self.theta_buf[s0:s1] if self.inplace else self.theta_buf[s0:s1].clone()
                self.comm.all_gather(self.theta_buf[b:e], src)
        return self.theta.flat

    # ---------------------------------------------------------------------------------------
    def bytes_reduced(self) -> int:
        """Metric bytes of one step on this rank: K_local x P x bytes per worker element."""
        return self.k_local * self.n * self.worker_bufs[0].element_size()

    def wire_bytes(self) -> int:
        """Bytes this rank sends over xGMI per step (ring/all-to-all lower bound)."""
        f = (self.world - 1) / self.world
        bg = self.theta_buf.element_size()
        wb = self.worker_bufs[0].element_size()
        if self.mode == "reduce":
            return int(f * self.n_pad * (4 + bg))
        return int(f * self.n_pad * (self.k_local * wb + (wb if self.broadcast == "workers" else bg)))


class PopulationCrossover:
    """EDT / SLERP children across GPUs: one population member per rank (member r on rank r,
    child c built on rank c). The only exchange is point-to-point: a grouped batch of RCCL
    send/recv delivers each child's parents to its rank (schedule.exchange_plan: one transfer per
    (member, destination), each over the direct xGMI link between the two GPUs); the merge itself
    is the single-GPU kernel, with no collective.

    The reference does this through the shared disk: every worker loads both parents' checkpoint
    directories (EDT_LM/train/crossover.py:255-258, EDT_EVOMERGE/train/crossover.py:167-168), and
    the RL master merges pairs one after another in one process (EDT_RL/edt.py:286-299)."""

    def __init__(self, layout: ParamLayout, dtype: torch.dtype, device, group=None, kernels=None,
                 comm: Collectives | None = None):
        self.comm = comm or TorchCollectives(group)
        self.world = self.comm.world
        self.rank = self.comm.rank
        self.kernels = kernels or _ops
        self.layout = layout
        self.device = device
        self.dtype = dtype
        self._bufs = {}
        self._plan = None

    def _buf(self, key, dtype=None):
        if key not in self._bufs:
            self._bufs[key] = torch.empty(self.layout.total, dtype=dtype or self.dtype, device=self.device)
        return self._bufs[key]

    def _exchange(self, pairs, payload, like=None):
        """payload(member, dst) -> tensors this rank ships for its member to the rank building
        child dst; like(src_member) -> the tensors this rank receives for that parent (shapes and
        dtypes; default: what this rank would ship for its own member). Returns the parents'
        tensor lists for this rank's child: ([...] of parent 1, [...] of parent 2)."""
        from .schedule import exchange_plan
        n = self.world
        if len(pairs) != n:
            raise ValueError(f"{len(pairs)} children for {n} ranks: one child per rank")
        plan = exchange_plan(pairs, list(range(n)), list(range(n)))
        mine = plan[self.rank]
        ops_ = []
        for m, dst in mine["send"]:
            for t in payload(m, dst):
                ops_.append(("send", t, dst))
        i, j = pairs[self.rank]
        got = {}
        for m, src in mine["recv"]:
            shapes = like(m) if like is not None else payload(self.rank, self.rank)
            bufs = [self._buf(("recv", m == i, k), t.dtype) for k, t in enumerate(shapes)]
            for b in bufs:
                ops_.append(("recv", b, src))
            got[m] = bufs
        self.comm.p2p(ops_)
        par1 = payload(i, self.rank) if i == self.rank else got[i]
        par2 = payload(j, self.rank) if j == self.rank else got[j]
        return par1, par2

    def slerp_step(self, member: torch.Tensor, pairs, t: torch.Tensor, out: torch.Tensor,
                   dot_threshold: float = 0.9995, eps: float = 1e-8) -> None:
        """SLERP child of pairs[rank] into `out` (EDT_RL/crossover.py:84-135 per Policy/Value;
        EDT_EVOMERGE/train/crossover.py:104-146). member: this rank's flat parameters."""
        (p1,), (p2,) = self._exchange(pairs, lambda m, dst: [member])
        if self._plan is None:
            self._plan = self.kernels.make_slerp_plan(self.layout.offsets, self.device)
        self.kernels.slerp_arena(self._plan, p1, p2, out, t, dot_threshold, eps)

    def pair_merge_step(self, base: torch.Tensor, trained: torch.Tensor, momentum: torch.Tensor | None,
                        pairs, out: torch.Tensor, out_momentum: torch.Tensor | None, lr: float = 0.7,
                        mu: float = 0.9, nesterov: bool = True, has_momentum: bool = True,
                        generation: int = 0) -> None:
        """EDT-LM child of pairs[rank] (EDT_LM/train/crossover.py:150-237): both parents ship
        (base, trained); the child inherits parent 1's outer momentum when parent 1 has one, else
        parent 2's (:183-227), and only that donor ships it. Which members have a momentum
        (`momentum is not None and has_momentum` on their rank) is agreed first, so every rank
        knows every message; a child with no donor past generation 0 raises NotImplementedError
        on every rank, as the reference's crossover does (:226-227)."""
        flags = self.comm.all_gather_object(bool(has_momentum and momentum is not None))
        donors = [i if flags[i] else (j if flags[j] else None) for i, j in pairs]
        if mu != 0 and generation > 0 and any(d is None for d in donors):
            raise NotImplementedError("Merging outer optimizer states not implemented for this case.")
        donor = donors[self.rank]
        if donor is not None and out_momentum is None:
            raise ValueError("the child inherits an outer momentum: pass out_momentum")

        def payload(m, dst):
            return [base, trained] + ([momentum] if donors[dst] == m else [])

        def like(m):
            return [base, trained] + ([out_momentum] if donor == m else [])
        par1, par2 = self._exchange(pairs, payload, like)
        if donor is not None:
            out_momentum.copy_((par1 if donor == pairs[self.rank][0] else par2)[2])
        self.kernels.pair_merge(par1[0], par2[0], par1[1], par2[1], out, out_momentum,
                                donor is not None, lr, mu, nesterov)
