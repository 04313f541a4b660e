"""The communicator seam of the multi-GPU schedules (distributed.py, population.py).

The schedules never call torch.distributed directly; they call one `Collectives` object:

  TorchCollectives    one process per GPU over torch.distributed ("nccl" = RCCL over xGMI on
                      ROCm; "gloo" in the CPU tests). Every blocking wait is bounded by
                      `timeout` (also handed to init_process_group by `init_torch`), so a dead
                      or stalled peer surfaces as `CommTimeout` instead of hanging the
                      generation forever — the reference's master polls its workers and gives
                      up on them (EDT_LM/diloco.py:46-71, diloco_sim.py:65-68).
  VirtualCollectives  N logical ranks inside ONE process (one thread each) sharing one device:
                      SURVEY.md §4's "virtual workers resident on one GPU". Each collective is a
                      rendezvous of the N threads; the last to arrive performs it as device
                      copies / fp32 sums on the (shared) current stream, in issue order after
                      every rank's producer kernels. It keeps RCCL's in-place conventions
                      (reduce-scatter output = the rank's slice of its input, all-gather input =
                      the rank's slice of its output), so the N-rank schedules — the bucket /
                      shard offsets, the all-to-all [dest][shard] layout, the n_pad tail — run
                      with the HIP kernels on one MI355X exactly as they are issued per rank.

Reference: the reference has no collectives — its "gather" is K x from_pretrained of the workers'
checkpoints and its "broadcast" K x save_pretrained (EDT_LM/diloco.py:231-235, 302-308).
"""
from __future__ import annotations

import copy
import datetime
import threading

import torch

from ._lib import EdtError


class CommTimeout(EdtError):
    """A collective or point-to-point exchange did not complete within the timeout (a peer
    died, hung, or issued a different collective)."""


class _Done:
    """The handle of a collective that is already enqueued in stream order."""

    def wait(self):
        return True


class _Works:
    """Several handles waited as one."""

    def __init__(self, works):
        self.works = works

    def wait(self):
        for w in self.works:
            w.wait()
        return True


class _TorchWork:
    """RCCL: wait() only orders the current stream after the collective (a host-blocking
    wait with a timeout would serialise the bucket pipeline); its timeout is the RCCL
    watchdog's, set by init_process_group (init_torch). gloo: a host wait bounded here."""

    def __init__(self, work, timeout, device_ordered=False):
        self.work, self.timeout, self.device_ordered = work, timeout, device_ordered

    def wait(self):
        try:
            ok = self.work.wait() if self.device_ordered else self.work.wait(self.timeout)
        except RuntimeError as e:          # gloo raises on timeout / a peer's failure
            raise CommTimeout(f"collective failed or timed out after {self.timeout}: {e}") from e
        if ok is False:
            raise CommTimeout(f"collective did not complete within {self.timeout}")
        return True


class Collectives:
    """Interface (see module docstring). `inplace`: the backend reduces/gathers in place
    (RCCL and the virtual ranks); otherwise the schedules stage through separate buffers."""
    world: int = 1
    rank: int = 0
    inplace: bool = False

    def reduce_scatter(self, out: torch.Tensor, inp: torch.Tensor, async_op: bool = False):
        raise NotImplementedError

    def all_gather(self, out: torch.Tensor, inp: torch.Tensor, async_op: bool = False):
        raise NotImplementedError

    def all_to_all(self, out: torch.Tensor, inp: torch.Tensor, async_op: bool = False):
        raise NotImplementedError

    def p2p(self, ops: list[tuple[str, torch.Tensor, int]], async_op: bool = False):
        """A grouped exchange: ("send" | "recv", tensor, peer rank); returns when all are done
        (stream-ordered for device backends), or with async_op a handle whose wait() orders the
        current stream after it (several exchanges can then be in flight at once)."""
        raise NotImplementedError

    def all_gather_object(self, obj) -> list:
        raise NotImplementedError

    def broadcast_object(self, obj, src: int = 0):
        raise NotImplementedError

    def barrier(self) -> None:
        raise NotImplementedError


DEFAULT_TIMEOUT = datetime.timedelta(minutes=10)


def init_torch(backend: str = "nccl", timeout: datetime.timedelta = DEFAULT_TIMEOUT, **kw) -> None:
    """init_process_group with the schedules' timeout (the RCCL watchdog aborts a communicator
    whose collective exceeds it, so a dead rank ends the run with an error)."""
    import torch.distributed as dist
    dist.init_process_group(backend, timeout=timeout, **kw)


class TorchCollectives(Collectives):
    def __init__(self, group=None, timeout: datetime.timedelta = DEFAULT_TIMEOUT):
        import torch.distributed as dist
        self.dist, self.group, self.timeout = dist, group, timeout
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        self.backend = dist.get_backend(group)
        self.inplace = self.backend == "nccl"

    def _ret(self, work, async_op):
        w = _TorchWork(work, self.timeout, self.inplace)
        if async_op:
            return w
        w.wait()
        return _Done()

    def reduce_scatter(self, out, inp, async_op=False):
        return self._ret(self.dist.reduce_scatter_tensor(out, inp, op=self.dist.ReduceOp.SUM, group=self.group,
                                                         async_op=True), async_op)

    def all_gather(self, out, inp, async_op=False):
        return self._ret(self.dist.all_gather_into_tensor(out, inp, group=self.group, async_op=True), async_op)

    def all_to_all(self, out, inp, async_op=False):
        return self._ret(self.dist.all_to_all_single(out, inp, group=self.group, async_op=True), async_op)

    def _global(self, r):
        return r if self.group is None else self.dist.get_global_rank(self.group, r)

    def p2p(self, ops, async_op=False):
        d = self.dist
        reqs = [d.P2POp(d.isend if kind == "send" else d.irecv, t, self._global(peer), self.group)
                for kind, t, peer in ops]
        works = [_TorchWork(w, self.timeout, self.inplace) for w in d.batch_isend_irecv(reqs)] if reqs else []
        handle = _Works(works)
        if async_op:
            return handle
        handle.wait()
        return _Done()

    def all_gather_object(self, obj):
        out = [None] * self.world
        self.dist.all_gather_object(out, obj, group=self.group)
        return out

    def broadcast_object(self, obj, src=0):
        box = [obj]
        self.dist.broadcast_object_list(box, src=self._global(src), group=self.group)
        return box[0]

    def barrier(self):
        self.dist.barrier(group=self.group)


# ------------------------------------------------------------------------------------------
# virtual ranks: N threads, one device

class VirtualWorld:
    """Shared state of N virtual ranks. `run(fn)` calls fn(comm) on N threads (comm =
    this world's VirtualCollectives for that rank) and returns their results in rank order; an
    exception on any rank breaks every rendezvous (the other ranks get CommTimeout instead of
    waiting forever) and is re-raised."""

    def __init__(self, world: int, timeout: float = 120.0):
        if world < 1:
            raise ValueError(world)
        self.world = world
        self.timeout = timeout
        self._barrier = threading.Barrier(world, timeout=timeout)
        self._slots = [None] * world
        self._result = None

    def comm(self, rank: int) -> "VirtualCollectives":
        return VirtualCollectives(self, rank)

    def rendezvous(self, rank: int, item, combine):
        """Every rank deposits `item`; one rank runs combine(items) once all have; every rank
        gets its result (or its exception)."""
        self._slots[rank] = item
        try:
            if self._barrier.wait() == 0:
                try:
                    self._result = ("ok", combine(list(self._slots)))
                except BaseException as e:            # noqa: BLE001 - handed to every rank
                    self._result = ("err", e)
            self._barrier.wait()
        except threading.BrokenBarrierError as e:
            raise CommTimeout(f"virtual rank {rank}: a peer failed or did not arrive within "
                              f"{self.timeout}s") from e
        kind, val = self._result
        if kind == "err":
            raise val
        return val

    def run(self, fn, devices=None):
        res = [None] * self.world
        errs = [None] * self.world

        def body(r):
            try:
                if devices is not None and torch.device(devices[r]).type == "cuda":
                    torch.cuda.set_device(torch.device(devices[r]))
                res[r] = fn(self.comm(r))
            except BaseException as e:                # noqa: BLE001
                errs[r] = e
                self._barrier.abort()

        ts = [threading.Thread(target=body, args=(r,), name=f"vrank{r}") for r in range(self.world)]
        for t in ts:
            t.start()
        for t in ts:
            t.join()
        first = next((e for e in errs if e is not None and not isinstance(e, CommTimeout)), None)
        first = first or next((e for e in errs if e is not None), None)
        if first is not None:
            raise first
        return res


def _slices(t: torch.Tensor, n: int):
    if t.numel() % n:
        raise EdtError(f"{t.numel()} elements do not split over {n} ranks")
    c = t.numel() // n
    return [t[r * c:(r + 1) * c] for r in range(n)]


class VirtualCollectives(Collectives):
    inplace = True

    def __init__(self, vw: VirtualWorld, rank: int):
        self.vw, self.rank, self.world = vw, rank, vw.world

    def _check(self, items, rel):
        n = self.world
        for out, inp in items:
            if out.dtype != inp.dtype or out.numel() * rel[0] != inp.numel() * rel[1]:
                raise EdtError("virtual collective: mismatched buffers")
            if out.numel() != items[0][0].numel():
                raise EdtError("virtual collective: ranks passed different sizes")

    def reduce_scatter(self, out, inp, async_op=False):
        def combine(items):
            self._check(items, (self.world, 1))
            ins = [_slices(i, self.world) for _, i in items]
            sums = []
            for r in range(self.world):              # every sum first: out_r may alias inp_r
                s = ins[0][r].clone()
                for k in range(1, self.world):
                    s.add_(ins[k][r])
                sums.append(s)
            for (o, _), s in zip(items, sums):
                o.copy_(s)
        self.vw.rendezvous(self.rank, (out, inp), combine)
        return _Done()

    def all_gather(self, out, inp, async_op=False):
        def combine(items):
            self._check(items, (1, self.world))
            srcs = [i.clone() for _, i in items]     # inp_r may alias out_r's r-th slice
            for o, _ in items:
                for dst, s in zip(_slices(o, self.world), srcs):
                    dst.copy_(s)
        self.vw.rendezvous(self.rank, (out, inp), combine)
        return _Done()

    def all_to_all(self, out, inp, async_op=False):
        def combine(items):
            self._check(items, (1, 1))
            srcs = [[s.clone() for s in _slices(i, self.world)] for _, i in items]
            for r, (o, _) in enumerate(items):
                for src, dst in enumerate(_slices(o, self.world)):
                    dst.copy_(srcs[src][r])
        self.vw.rendezvous(self.rank, (out, inp), combine)
        return _Done()

    def p2p(self, ops, async_op=False):
        for kind, _, peer in ops:
            if kind not in ("send", "recv") or not 0 <= peer < self.world:
                raise EdtError(f"bad p2p op {kind} to {peer}")

        def combine(items):
            sends = {}
            for r, ops_r in enumerate(items):
                for kind, t, peer in ops_r:
                    if kind == "send":
                        sends.setdefault((r, peer), []).append(t.clone())
            for r, ops_r in enumerate(items):
                for kind, t, peer in ops_r:
                    if kind == "recv":
                        q = sends.get((peer, r))
                        if not q:
                            raise EdtError(f"virtual p2p: rank {r} receives from {peer}, which sends nothing")
                        s = q.pop(0)
                        if s.numel() != t.numel() or s.dtype != t.dtype:
                            raise EdtError(f"virtual p2p {peer}->{r}: {s.numel()} {s.dtype} into {t.numel()} {t.dtype}")
                        t.copy_(s)
            left = [k for k, q in sends.items() if q]
            if left:
                raise EdtError(f"virtual p2p: unmatched sends {left}")
        self.vw.rendezvous(self.rank, list(ops), combine)
        return _Done()

    def all_gather_object(self, obj):
        return copy.deepcopy(self.vw.rendezvous(self.rank, obj, lambda items: list(items)))

    def broadcast_object(self, obj, src=0):
        got = self.vw.rendezvous(self.rank, obj, lambda items: items[src])
        return got if self.rank == src else copy.deepcopy(got)   # a process would unpickle a copy

    def barrier(self):
        self.vw.rendezvous(self.rank, None, lambda items: None)
