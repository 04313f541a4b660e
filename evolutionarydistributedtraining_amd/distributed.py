"""DiLoCo outer step across GPUs: one process per GPU, RCCL over xGMI (torch.distributed "nccl").

The reference has no collectives: its "gather" is K x `from_pretrained` of the workers'
checkpoints on a shared disk and its "broadcast" is K x `save_pretrained` (EDT_LM/diloco.py:
231-235, 302-308). Here the population is resident in HBM across the node and the cross-replica
mean is a real exchange step. Three schedules, all bucketed so RCCL traffic on the comm stream
overlaps the HBM-bound kernels on the compute stream:

  mode="reduce"          each rank fuses its local workers into an fp32 partial sum
                         (edt_delta_partial), reduce-scatter(sum, fp32) -> SGD on the owned shard
                         (momentum sharded 1/N, edt_sgd_apply) -> all-gather of theta. Wire bytes
                         per rank and step: (N-1)/N * P * (4 + b_g). The cross-rank sum is RCCL's
                         (its order depends on the algorithm RCCL picks); within DESIGN §3's bound of
                         the reference's sequential order.
  mode="reduce_ordered"  the same partials, an all-to-all of them instead of the reduce-scatter,
                         then edt_sgd_apply_sum: the owned shard's N partials summed in rank order
                         + SGD. Same wire bytes as reduce; one fixed summation order whatever RCCL
                         does (reproducible run to run, bit-exact with the oracle's split).
  mode="exact"           all-to-all of the raw worker shards to their owners, then the single-GPU
                         fused kernel on each shard (the reference's worker order, bit-exact),
                         all-gather of theta. Wire bytes: (N-1)/N * P * (K_local * b_w + b_g).
  broadcast              what the all-gather delivers to every rank. "theta": the full master
                         replica (theta's dtype). "workers" (exact mode only): the new theta rounded
                         to the worker dtype, straight into every local worker arena — the start of
                         the next inner loop, which is all the reference ships to the workers
                         (diloco.py:302-308 saves the base to every worker dir; the bf16 workers load
                         it rounded). The fp32 master then stays sharded (`gather_theta()` assembles
                         it on demand, e.g. for a checkpoint). Wire bytes: (N-1)/N * P * (K_local + 1) * b_w.
  mode="auto" / broadcast="auto" (defaults) pick the combination with the fewest wire bytes,
  ties to exact, then reduce_ordered: at K = 8 bf16 workers, fp32 theta: N = 2 reduce_ordered/theta
  (8 B/elem), N = 4 and 8 exact/workers (6 and 4 B/elem); all fp32: N = 2 and 4 reduce_ordered,
  N = 8 exact.

Every rank holds 1/N of the momentum and owns contiguous shards of every bucket.
"""
from __future__ import annotations

import math

import torch

from . import ops as _ops
from ._lib import EdtError
from .collectives import Collectives, TorchCollectives
from .diloco import check_sgd_hparams
from .params import ParamArena, ParamLayout
from .tracing import trange, traced


def _timing_event():
    return torch.cuda.Event(enable_timing=True)


class ShardedOuterSync:
    def __init__(self, layout: ParamLayout, theta_dtype: torch.dtype, worker_dtype: torch.dtype,
                 k_local: int, device, lr: float = 0.7, momentum: float = 0.9, nesterov: bool = True,
                 mode: str = "auto", bucket_elems: int = 1 << 26, group=None, kernels=None,
                 broadcast: str = "auto", comm: Collectives | None = None,
                 cpu_tails: tuple[int, int] | None = None):
        if mode not in ("reduce", "reduce_ordered", "exact", "auto") or broadcast not in ("theta", "workers", "auto"):
            raise ValueError((mode, broadcast))
        if mode.startswith("reduce") and broadcast == "workers":
            raise ValueError("the reduce schedules need the full theta replica (broadcast='theta')")
        check_sgd_hparams(lr, momentum, nesterov)
        # the communicator seam: torch.distributed (RCCL / gloo) by default, or N virtual ranks
        # on one device (collectives.VirtualWorld)
        self.comm = comm or TorchCollectives(group)
        self.world = self.comm.world
        self.rank = self.comm.rank
        wb = torch.empty(0, dtype=worker_dtype).element_size()
        gb = torch.empty(0, dtype=theta_dtype).element_size()
        cands = {("reduce", "theta"): 4 + gb, ("reduce_ordered", "theta"): 4 + gb,
                 ("exact", "theta"): k_local * wb + gb, ("exact", "workers"): (k_local + 1) * wb}
        cands = {key: v for key, v in cands.items()
                 if mode in ("auto", key[0]) and broadcast in ("auto", key[1])}
        # fewest wire bytes per element; ties go to the bit-exact schedule, then to the one whose
        # cross-rank sum has a fixed order (reduce_ordered) over RCCL's own (reduce)
        pref = {"exact": 0, "reduce_ordered": 1, "reduce": 2}
        mode, broadcast = min(cands, key=lambda key: (cands[key], pref[key[0]], key[1] != "workers"))
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
        self.event_factory = _timing_event   # bench.py's host rehearsal swaps in host-clock events
        # (Vec::size(), threads) of the reference's host: exact mode reproduces its bf16 scalar tails
        # (diloco.outer_step's cpu_tails; the reduce mode reassociates the sum anyway)
        self.tail_bits = None
        if cpu_tails is not None and mode == "exact" and self.kernels is _ops:
            from .torchcompat import torch_cpu_tail_bits
            self.tail_bits = torch_cpu_tail_bits(list(layout.numels) + [self.n_pad - n], vec_elems=cpu_tails[0],
                                                 num_threads=cpu_tails[1], device=device)
        if mode == "reduce":
            self.acc = torch.zeros(self.n_pad, dtype=torch.float32, device=device)
            self.acc_shard = None if self.inplace else torch.empty(shard_total, dtype=torch.float32, device=device)
        elif mode == "reduce_ordered":
            # partials laid out [dest rank][shard] per bucket, received as [src rank][shard]
            self.acc = torch.zeros(self.n_pad, dtype=torch.float32, device=device)
            self.acc_recv = torch.zeros(self.n_pad, dtype=torch.float32, device=device)
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
        a, b = self.event_factory(), self.event_factory()
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
        if self.mode == "reduce_ordered":
            return self.n_pad * (self.k_local * wb + gb + 4) + shard * (4 * self.world + 2 * gb + mom)
        return self.n_pad * (self.k_local * wb + gb + 4) + shard * (4 + 2 * gb + mom)

    @traced("edt/ShardedOuterSync.step")
    def step(self) -> None:
        """One outer step; returns when the work is enqueued (stream-ordered, async)."""
        with trange(f"edt/sharded.{self.mode}/{self.broadcast}"):
            self._step_body()

    def _step_body(self) -> None:
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
        elif self.mode == "reduce_ordered":
            # phase 1: local partials, each bucket's all-to-all as soon as it is ready (the partial
            # of bucket [b, e) is laid out [dest rank][shard]; it arrives as [src rank][shard])
            works = []
            for b, e in self.buckets:
                self._launch(k.delta_partial, self.theta_buf[b:e], [w[b:e] for w in self.worker_bufs],
                             self.k_total, self.acc[b:e], False)
                works.append(self.comm.all_to_all(self.acc_recv[b:e], self.acc[b:e], async_op=True))
            # phase 2: the owned shard's N partials summed in rank order + SGD, then the all-gather
            for (b, e), w in zip(self.buckets, works):
                w.wait()
                s0, s1 = self._shard(b, e)
                per = s1 - s0
                parts = list(self.acc_recv[b:e].view(self.world, per))
                mom = None if self.mom_shard is None else self.mom_shard[mom_off:mom_off + per]
                self._launch(self._sgd_sum, self.theta_buf[s0:s1], parts, mom)
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
                fused = self.broadcast == "workers" and k is _ops and self.tail_bits is None
                if self.tail_bits is not None:     # shards start at multiples of 64: whole bytes
                    import functools
                    fn = functools.partial(k.outer_step, tail_bits=self.tail_bits[s0 // 8:(s1 + 7) // 8])
                else:
                    fn = k.outer_step
                self._launch(fn, self.theta_buf[s0:s1], shards, mom, self.has_momentum, self.lr,
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

    def _sgd_sum(self, theta, parts, mom):
        """SGD from the shard's per-rank partials, summed in rank order."""
        k = self.kernels
        if hasattr(k, "sgd_apply_sum"):
            k.sgd_apply_sum(theta, parts, mom, self.has_momentum, self.lr, self.momentum, self.nesterov)
            return
        total = parts[0].clone()             # stand-in kernels (CPU tests): the same order in torch
        for p in parts[1:]:
            total.add_(p)
        k.sgd_apply(theta, total, mom, self.has_momentum, self.lr, self.momentum, self.nesterov)

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
        if self.mode.startswith("reduce"):
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

    @traced("edt/PopulationCrossover.slerp_step")
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


class ShardedPopulationCrossover:
    """A generation of a population of P = world members (one per GPU: BASELINE configs[4], the
    EDT-RL / EVOMERGE population of 8 SLERP-crossed on 7B bodies across 8 GPUs; or the EDT-LM pair
    merges), link-balanced. PopulationCrossover ships each child's two parents whole to the child's
    rank — two full members over at most two of the GPU's seven xGMI links. Here every rank owns a
    parameter-index shard instead (a contiguous range of whole SLERP chunks, ~1/N of the layout):

      1. members -> shards: rank r sends rank s the slice of its member in s's range (grouped p2p,
         every link busy: (N-1)/N of a member out and in per rank);
      2. SLERP: per chunk of the rank's range the sums the generation needs — each distinct
         parent's norm and each distinct dot its children use, per connected component of the
         pair graph (edt_slerp_needed_sums: edt_slerp_population's needed-sums pass, r5; a
         component's row is its D norms, D ring-dot and <= 4 chord slots, against the Gram
         triangle's 36 at N = 8) — the table rows all-gathered
         (nchunks x those sums doubles: 12-16 MB at 7B for a roulette-drawn generation, against ~31 MB
         for the triangle), then every child's coefficients (edt_slerp_needed_coef) — each chunk's
         sums come from the same kernel in the same order wherever the chunk lives, so every child
         is bit-identical to edt_slerp_merge on its two parents; then the rank's range of every
         child (edt_slerp_blend_children).
         EDT-LM: the rank's range of every child (edt_pair_merge_population), nothing to gather;
      3. child shards -> children: the range of child c goes to rank c.

    Wire bytes per rank and generation: (N-1)/N x (member + child) (+ the donor momenta for
    EDT-LM), spread over all N-1 links, against up to two whole members over one or two links.
    Reference: EDT_RL/edt.py:286-299 (the master merges pair after pair), EDT_EVOMERGE/edt.py:262-280.
    A rank's range starts at a multiple of 8 elements below its first chunk (<= 7 elements shared
    with the previous rank), so every chunk keeps its vector alignment and hence its sums.

    groups > 1 (SLERP): every rank's range is cut into that many groups of whole chunks and the
    exchanges run per group, all of a phase's groups in flight at once: the Gram pass of group g
    starts as soon as g's member slices have landed (while later groups are still on the links),
    and group g of the children leaves as soon as its blend is done (while later groups blend).
    Same bytes, same kernels on the same chunks: the children are bit-identical to groups = 1."""

    def __init__(self, layout: ParamLayout, dtype: torch.dtype, device, kind: str = "slerp",
                 out_dtype: torch.dtype | None = None, comm: Collectives | None = None, group=None,
                 kernels=None, chunk_elems: int = 1 << 16, groups: int = 1):
        if kind not in ("slerp", "sgd"):
            raise ValueError(kind)
        self.comm = comm or TorchCollectives(group)
        self.world, self.rank = self.comm.world, self.comm.rank
        if self.world > 8 and kind == "slerp":
            raise ValueError("the Gram pass takes at most 8 members (one per rank)")
        if self.world > 16:
            raise ValueError("at most 16 children per launch")
        self.kind, self.layout, self.device = kind, layout, torch.device(device)
        self.dtype, self.out_dtype = dtype, out_dtype or dtype
        self.kernels = kernels or _ops
        import numpy as np
        self.plan = self.kernels.make_slerp_plan(layout.offsets, self.device, chunk_elems=chunk_elems)
        host = np.asarray(self.plan.chunks_host, dtype=np.int64).reshape(-1, 3)
        n, N = layout.total, self.world
        starts = host[:, 0] if len(host) else np.zeros(0, dtype=np.int64)
        cuts = [0] + [int(np.searchsorted(starts, (r * n) // N, side="left")) for r in range(1, N)] + [len(host)]
        self.ranges = []           # per rank: (first chunk, end chunk, base, start, end) in elements
        for r in range(N):
            c0, c1 = cuts[r], max(cuts[r], cuts[r + 1])
            if c1 > c0:
                start, end = int(host[c0, 0]), int(host[c1 - 1, 0] + host[c1 - 1, 1])
            else:
                start = end = int(host[c0, 0]) if c0 < len(host) else n
            self.ranges.append((c0, c1, start // 8 * 8, start, end))
        if groups < 1:
            raise ValueError(groups)
        # per rank: its chunk range in `groups` contiguous groups (fewer when it has fewer chunks),
        # each (first chunk, end chunk, lo, hi) with [lo, hi) the elements a group carries: the
        # first group from the rank's aligned base, the others from their first chunk's start
        self.granges = []
        for r in range(N):
            a, b, rbase = self.ranges[r][0], self.ranges[r][1], self.ranges[r][2]
            G = min(groups, b - a)
            gl = []
            for g in range(G):
                g0, g1 = a + (b - a) * g // G, a + (b - a) * (g + 1) // G
                lo = rbase if g == 0 else int(host[g0, 0])
                gl.append((g0, g1, lo, int(host[g1 - 1, 0] + host[g1 - 1, 1])))
            self.granges.append(gl)
        self.groups = groups
        c0, c1, base, start, end = self.ranges[self.rank]
        self.nloc = c1 - c0
        self.base, self.start, self.end = base, start, end
        loc = host[c0:c1].copy()
        loc[:, 0] -= base
        self.local_chunks = torch.from_numpy(loc).to(self.device) if self.device.type == "cuda" else torch.from_numpy(loc)
        L = end - base
        self._shard_len = max(L, 8)     # no closure over self: the buffers go with the object
        self._bufs = {}

    def _buf(self, key, dt):
        if key not in self._bufs:
            self._bufs[key] = torch.empty(self._shard_len, dtype=dt, device=self.device)
        return self._bufs[key]

    def _scatter(self, tensors, tag):
        """Every rank's tensors -> this rank's range of each: {tag, j: buffer of rank j's tensor}."""
        ops_, got = [], {}
        L = self.end - self.base
        for s in range(self.world):
            _, _, b, _, e = self.ranges[s]
            if s != self.rank and e > b:
                for i, t in enumerate(tensors):
                    ops_.append(("send", t[b:e], s))
        for j in range(self.world):
            bufs = [self._buf((tag, i, j), t.dtype) for i, t in enumerate(tensors)]
            got[j] = [bb[:L] for bb in bufs]
            if j == self.rank:
                for bb, t in zip(got[j], tensors):
                    bb.copy_(t[self.base:self.end])
            elif L > 0:
                ops_.extend(("recv", bb, j) for bb in got[j])
        self.comm.p2p(ops_)
        return got

    def _gather_children(self, shards, outs):
        """Child q's range from every rank into outs (this rank's child): shards[q] = this rank's
        range of child q (buffers of base..end); outs = this rank's child tensors."""
        ops_ = []
        off = self.start - self.base
        for q in range(self.world):
            for sh, out in zip(shards[q], outs):
                if q == self.rank:
                    out[self.start:self.end].copy_(sh[off:self.end - self.base])
                elif self.end > self.start:
                    ops_.append(("send", sh[off:self.end - self.base], q))
        for j in range(self.world):
            _, _, _, st, en = self.ranges[j]
            if j != self.rank and en > st:
                ops_.extend(("recv", out[st:en], j) for out in outs)
        self.comm.p2p(ops_)

    def _scatter_groups(self, member, tag):
        """_scatter of one tensor, one grouped exchange per chunk group, all issued at once.
        Returns (buffers per rank j, one handle per group)."""
        L = self.end - self.base
        got = {j: self._buf((tag, 0, j), member.dtype)[:L] for j in range(self.world)}
        mine = self.granges[self.rank]
        handles = []
        for g in range(self.groups):
            ops_ = []
            for s_ in range(self.world):
                if s_ != self.rank and g < len(self.granges[s_]):
                    _, _, lo, hi = self.granges[s_][g]
                    ops_.append(("send", member[lo:hi], s_))
            if g < len(mine):
                _, _, lo, hi = mine[g]
                ops_.extend(("recv", got[j][lo - self.base:hi - self.base], j)
                            for j in range(self.world) if j != self.rank)
            handles.append(self.comm.p2p(ops_, async_op=True))
        got[self.rank].copy_(member[self.base:self.end])
        return got, handles

    def _gather_group(self, g, outs, out):
        """Group g of this rank's range of every child q to rank q, and group g of every other
        rank's range of this rank's child into `out` (issued, not waited)."""
        ops_ = []
        mine = self.granges[self.rank]
        if g < len(mine):
            _, _, lo, hi = mine[g]
            lo = max(lo, self.start)
            for q in range(self.world):
                if q == self.rank:
                    out[lo:hi].copy_(outs[q][lo - self.base:hi - self.base])
                else:
                    ops_.append(("send", outs[q][lo - self.base:hi - self.base], q))
        for j in range(self.world):
            if j != self.rank and g < len(self.granges[j]):
                _, _, lo, hi = self.granges[j][g]
                lo = max(lo, self.ranges[j][3])
                ops_.append(("recv", out[lo:hi], j))
        return self.comm.p2p(ops_, async_op=True)

    def _reference_dots(self, members, pairs, t, dots, dot_threshold, eps, ref):
        """Reference-dot mode of the sharded generation (ops.RefDot): the reference's fp32 dot of
        every flagged (child, segment) — the BLAS sdot chains and numpy's pairwise sum run over the
        WHOLE segment in order, so each segment is computed by the rank that holds its first chunk:
        from its own shards when the segment ends in its range, else after the later ranks send it
        the rest of that segment of the parents it needs (only segments that straddle a range
        boundary: at most N - 1). The values are all-gathered (host objects) and every rank forms
        the reference's coefficients of every child from them (ops.reference_coefficients): the
        children equal the reference's merges bit for bit with band < 0. Returns (coef [Q, nseg, 2],
        dots [Q, nseg]) on the device."""
        import numpy as np
        ref.check_host()
        k, N, Q = self.kernels, self.world, len(pairs)
        plan, nseg = self.plan, self.plan.nseg
        host = np.asarray(plan.chunks_host, dtype=np.int64).reshape(-1, 3)
        first = np.searchsorted(host[:, 2], np.arange(nseg + 1), side="left") if len(host) \
            else np.zeros(nseg + 1, dtype=np.int64)
        d = dots[:Q, :nseg].detach().cpu().numpy().astype(np.float32)
        if ref.band < 0:
            flag = np.ones((Q, nseg), dtype=bool)
        else:                               # refdot_flag_kernel's test, in fp32
            flag = np.abs(np.abs(d) - np.float32(dot_threshold)) <= np.float32(ref.band)
        flag &= (first[1:] > first[:-1])[None, :]          # segments with elements
        owner = np.full(nseg, -1, dtype=np.int64)
        for r in range(N):
            a, b = self.ranges[r][:2]
            owner[(first[:-1] >= a) & (first[:-1] < b)] = r
        c0, c1 = self.ranges[self.rank][:2]
        dt = members[0].dtype
        # 1. the rest of each straddling flagged segment to its owner (same op order on every rank)
        ops_, bufs = [], {}
        for s in range(nseg):
            r = int(owner[s])
            if r < 0 or not flag[:, s].any() or first[s + 1] <= self.ranges[r][1]:
                continue
            need = sorted({int(x) for q in range(Q) if flag[q, s] for x in pairs[q]})
            seg_lo = int(host[first[s], 0])
            seg_hi = int(host[first[s + 1] - 1, 0] + host[first[s + 1] - 1, 1])
            if r == self.rank:
                own_hi = int(host[c1 - 1, 0] + host[c1 - 1, 1])
                for m in need:
                    buf = bufs[(s, m)] = torch.empty(seg_hi - seg_lo, dtype=dt, device=self.device)
                    buf[:own_hi - seg_lo].copy_(members[m][seg_lo - self.base:own_hi - self.base])
            for j in range(N):
                if j == r:
                    continue
                ja, jb, jbase = self.ranges[j][:3]
                lo, hi = max(int(first[s]), ja), min(int(first[s + 1]), jb)
                if hi <= lo:
                    continue
                elo, ehi = int(host[lo, 0]), int(host[hi - 1, 0] + host[hi - 1, 1])
                for m in need:
                    if j == self.rank:
                        ops_.append(("send", members[m][elo - jbase:ehi - jbase], r))
                    elif r == self.rank:
                        ops_.append(("recv", bufs[(s, m)][elo - seg_lo:ehi - seg_lo], j))
        if ops_:
            self.comm.p2p(ops_)
        # 2. this rank's segments: whole ones from its shards (one pass per child), straddling ones
        #    from the assembled buffers
        mine = owner == self.rank
        whole = mine & (first[1:] <= c1)
        sf = torch.from_numpy(np.clip(first - c0, 0, max(0, c1 - c0)).astype(np.int32)).to(self.device)
        found = []
        for q, (i, j) in enumerate(pairs):
            fq = flag[q] & whole
            if fq.any():
                val = k.slerp_refdot(members[i], members[j], self.local_chunks, sf, nseg, plan.chunk_elems,
                                     torch.from_numpy(fq.astype(np.int32)).to(self.device), ref, eps)
                vh = val[:nseg].cpu().numpy()
                found.extend((q, int(s), float(vh[s])) for s in np.nonzero(fq)[0])
        for s in sorted({s for (s, _) in bufs}):
            seg_len = int(host[first[s + 1] - 1, 0] + host[first[s + 1] - 1, 1] - host[first[s], 0])
            ce = plan.chunk_elems
            rows = np.asarray([(x, min(ce, seg_len - x), 0) for x in range(0, seg_len, ce)], dtype=np.int64)
            ch = torch.from_numpy(rows).to(self.device)
            sf1 = torch.tensor([0, len(rows)], dtype=torch.int32).to(self.device)
            one = torch.ones(1, dtype=torch.int32).to(self.device)
            for q, (i, j) in enumerate(pairs):
                if flag[q, s]:
                    val = k.slerp_refdot(bufs[(s, i)], bufs[(s, j)], ch, sf1, 1, ce, one, ref, eps)
                    found.append((q, int(s), float(val[:1].cpu().numpy()[0])))
        # 3. every rank: all values, then the reference's coefficients of every child
        final = d.copy()
        for part in self.comm.all_gather_object(found):
            for q, s, v in part:
                final[q, s] = np.float32(v)
        from .ops import reference_coefficients
        coef = reference_coefficients(final, t[:nseg].detach().cpu().numpy(), dot_threshold)
        return torch.from_numpy(coef).to(self.device), torch.from_numpy(final).to(self.device)

    @traced("edt/ShardedPopulationCrossover.slerp_step")
    def slerp_step(self, member: torch.Tensor, pairs, t: torch.Tensor, out: torch.Tensor,
                   dot_threshold: float = 0.9995, eps: float = 1e-8, ref_dot=None) -> torch.Tensor:
        """Child pairs[rank] into `out`; returns the per-segment dots of every child [N, nseg].
        ref_dot (ops.RefDot): the reference-dot mode (_reference_dots; the groups > 1 pipeline is
        not used in that mode: the coefficients need every rank's values first)."""
        if len(pairs) != self.world:
            raise ValueError(f"{len(pairs)} children for {self.world} ranks")
        k, N = self.kernels, self.world
        layout = k.needed_table(pairs, N, self.plan.nchunks)
        table = self._bufs.get("needed")
        if table is None or table.numel() < max(1, layout.doubles):
            table = self._bufs["needed"] = torch.empty(max(1, layout.doubles), dtype=torch.float64, device=self.device)
        c0, c1 = self.ranges[self.rank][:2]
        mine = self.granges[self.rank]
        if self.groups > 1 and ref_dot is None:
            sh, handles = self._scatter_groups(member, "m")
            members = [sh[j] for j in range(N)]
            for g, h in enumerate(handles):
                h.wait()
                if g < len(mine):
                    g0, g1 = mine[g][0] - c0, mine[g][1] - c0
                    k.slerp_needed_sums(members, layout, self.local_chunks[g0:g1], g1 - g0, table, c0 + g0)
        else:
            sh = self._scatter([member], "m")
            members = [sh[j][0] for j in range(N)]
            if self.nloc:
                k.slerp_needed_sums(members, layout, self.local_chunks, self.nloc, table, c0)
        ops_ = []                       # all-gather of the table rows: every rank's chunk range, per block
        for b in range(len(layout.blocks)):
            for s in range(N):
                if s != self.rank and self.nloc:
                    ops_.append(("send", layout.rows(table, b, c0, c1), s))
            for j in range(N):
                ja, jb = self.ranges[j][:2]
                if j != self.rank and jb > ja:
                    ops_.append(("recv", layout.rows(table, b, ja, jb), j))
        self.comm.p2p(ops_)
        coef, dots = k.slerp_needed_coef(self.plan, table, layout, t, dot_threshold, eps)
        if ref_dot is not None:
            coef, dots = self._reference_dots(members, pairs, t, dots, dot_threshold, eps, ref_dot)
        outs = [self._buf(("c", q), self.out_dtype)[:self.end - self.base] for q in range(N)]
        if self.groups > 1 and ref_dot is None:
            handles = []
            for g in range(self.groups):
                if g < len(mine):
                    g0, g1 = mine[g][0] - c0, mine[g][1] - c0
                    k.slerp_blend_children(members, pairs, outs, self.local_chunks[g0:g1], g1 - g0, coef,
                                           self.plan.nseg)
                handles.append(self._gather_group(g, outs, out))
            for h in handles:
                h.wait()
            return dots
        if self.nloc:
            k.slerp_blend_children(members, pairs, outs, self.local_chunks, self.nloc, coef, self.plan.nseg)
        self._gather_children([[o] for o in outs], [out])
        return dots

    def pair_merge_step(self, base: torch.Tensor, trained: torch.Tensor, momentum: torch.Tensor | None,
                        pairs, out: torch.Tensor, out_momentum: torch.Tensor | None, lr: float = 0.7,
                        mu: float = 0.9, nesterov: bool = True, has_momentum: bool = True,
                        generation: int = 0) -> None:
        """EDT-LM child pairs[rank] into out / out_momentum (EDT_LM/train/crossover.py:150-237;
        donor = parent 1 when it has an outer momentum, else parent 2, as PopulationCrossover)."""
        if len(pairs) != self.world:
            raise ValueError(f"{len(pairs)} children for {self.world} ranks")
        # each rank's momentum flag and the dtypes its momentum buffers would travel in: every rank
        # sizes its p2p buffers from its own send list, so a dtype that differs across ranks would
        # post sends and receives of different byte counts — refused on every rank instead
        has = bool(has_momentum and momentum is not None)
        mdt = str(out_momentum.dtype) if out_momentum is not None else None
        info = self.comm.all_gather_object((has, mdt, str(momentum.dtype) if has else None))
        flags = [f for f, _, _ in info]
        donors = [i if flags[i] else (j if flags[j] else None) for i, j in pairs]
        if mu != 0 and generation > 0 and any(d is None for d in donors):
            raise NotImplementedError("Merging outer optimizer states not implemented for this case.")
        send_mom = any(d is not None for d in donors)      # some child inherits a buffer
        if send_mom and any(m is None for _, m, _ in info):     # on every rank, not just the one missing it
            raise ValueError("the child inherits an outer momentum: pass out_momentum on every rank")
        if send_mom and (len({m for _, m, _ in info}) != 1 or any(d not in (None, info[0][1]) for _, _, d in info)):
            raise EdtError(f"outer momentum dtypes differ across ranks or from the child's: {info}")
        with_mom = out_momentum is not None                # children write one (mu != 0)
        stand_in = (lambda: torch.zeros_like(base, dtype=out_momentum.dtype)) if send_mom else None
        send = [base, trained] + ([momentum if has else stand_in()] if send_mom else [])
        sh = self._scatter(send, "p")
        L = self.end - self.base
        children = []
        outs = [[self._buf(("c", q), self.out_dtype)[:L]] + ([self._buf(("cm", q), out_momentum.dtype)[:L]]
                                                             if with_mom else []) for q in range(self.world)]
        for q, (i, j) in enumerate(pairs):
            d = donors[q]
            children.append({"b1": sh[i][0], "b2": sh[j][0], "m1": sh[i][1], "m2": sh[j][1], "out": outs[q][0],
                             "momentum": outs[q][1] if with_mom else None,
                             "momentum_in": sh[d][2] if d is not None else None, "has_momentum": d is not None})
        if L > 0:
            self.kernels.pair_merge_population(children, lr, mu, nesterov)
        self._gather_children(outs, [out] + ([out_momentum] if with_mom else []))
