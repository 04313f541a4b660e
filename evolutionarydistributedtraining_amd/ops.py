"""Flat-buffer operators: one call = one fused HIP launch over a whole parameter arena.

Every function takes device-resident, contiguous tensors (flat views of the population's
parameter arenas, see `params.ParamArena`) and launches on the current HIP stream. Nothing here
synchronises, allocates persistent memory or falls back to the CPU: a missing library or device
raises `EdtError`.
"""
from __future__ import annotations

import ctypes
import threading
from dataclasses import dataclass

import torch

from . import _lib as L


def outer_step(theta: torch.Tensor, workers: list[torch.Tensor], momentum: torch.Tensor | None,
               has_momentum: bool, lr: float, momentum_coef: float, nesterov: bool,
               broadcast: list[torch.Tensor] | None = None, tail_bits: torch.Tensor | None = None) -> None:
    """Fused DiLoCo outer step (EDT_LM/diloco.py:238-289): theta and momentum updated in place.

    theta: flat float32/bfloat16; workers: K flat tensors of one dtype (K > 64: chained launches
    through a scratch running sum); momentum: flat, theta's dtype (required when momentum_coef != 0).
    broadcast: buffers of the workers' dtype (may be the workers themselves) that receive the new
    theta rounded to that dtype in the same pass (edt_outer_step_bcast: the broadcast of
    diloco.py:302-308 fused into the step, no re-read of theta per copy).
    tail_bits: torchcompat.torch_cpu_tail_bits of the reference's host (uint8 device bitmask of the
    arena): bf16 elements on torch CPU's scalar tails round add(alpha) twice, as the reference does
    there (edt_outer_step_tail); with a broadcast too, the tail step runs and then each broadcast
    buffer is copied from theta."""
    lib = L.lib()
    if not workers:
        raise L.EdtError("no workers")
    L.require_device(theta, momentum, *workers, *(broadcast or []))
    n = theta.numel()
    for w in workers:
        if w.numel() != n or w.dtype != workers[0].dtype:
            raise L.EdtError("every worker buffer must match theta's size and share one dtype")
    if momentum is not None and (momentum.numel() != n or momentum.dtype != theta.dtype):
        raise L.EdtError("momentum must have theta's size and dtype")
    if broadcast and any(b.numel() != n or b.dtype != workers[0].dtype for b in broadcast):
        raise L.EdtError("broadcast buffers must match theta's size and the workers' dtype")
    if tail_bits is not None:
        # checked first: the tail emulation is never dropped because a broadcast was asked for
        L.require_device(tail_bits)
        if len(workers) > L.EDT_MAX_WORKERS:
            raise L.EdtError("tail emulation runs in the plain fused step (<= 64 workers)")
        if tail_bits.dtype != torch.uint8 or tail_bits.numel() * 8 < n:
            raise L.EdtError("tail_bits: uint8 with one bit per element")
        L.check(lib.edt_outer_step_tail(L.ptr(theta), L.dtype_code(theta), L.ptr_array(workers),
                                        L.dtype_code(workers[0]), len(workers), L.ptr(momentum),
                                        int(has_momentum), n, float(lr), float(momentum_coef), int(nesterov),
                                        L.ptr(tail_bits), L.stream_ptr(theta.device)), "edt_outer_step_tail")
        for b in broadcast or []:          # the broadcast after the step, as diloco._step_flat does
            b.copy_(theta)
        return
    if broadcast:
        if len(workers) <= L.EDT_MAX_WORKERS and len(broadcast) <= L.EDT_MAX_WORKERS:
            L.check(lib.edt_outer_step_bcast(L.ptr(theta), L.dtype_code(theta), L.ptr_array(workers),
                                             L.dtype_code(workers[0]), len(workers), L.ptr(momentum),
                                             int(has_momentum), n, float(lr), float(momentum_coef),
                                             int(nesterov), L.ptr_array(broadcast), len(broadcast),
                                             L.stream_ptr(theta.device)), "edt_outer_step_bcast")
            return
        outer_step(theta, workers, momentum, has_momentum, lr, momentum_coef, nesterov)
        for b in broadcast:
            b.copy_(theta)
        return
    if len(workers) <= L.EDT_MAX_WORKERS:
        L.check(lib.edt_outer_step(L.ptr(theta), L.dtype_code(theta), L.ptr_array(workers),
                                   L.dtype_code(workers[0]), len(workers), L.ptr(momentum),
                                   int(has_momentum), n, float(lr), float(momentum_coef),
                                   int(nesterov), L.stream_ptr(theta.device)), "edt_outer_step")
        return
    ws = torch.empty_like(theta)
    L.check(lib.edt_outer_step_ws(L.ptr(theta), L.dtype_code(theta), L.ptr_array(workers),
                                  L.dtype_code(workers[0]), len(workers), L.ptr(momentum),
                                  int(has_momentum), n, float(lr), float(momentum_coef), int(nesterov),
                                  L.ptr(ws), L.stream_ptr(theta.device)), "edt_outer_step_ws")


def outer_step_list(thetas: list[torch.Tensor], workers: list[list[torch.Tensor]],
                    momenta: list[torch.Tensor] | None, has_momentum: bool, lr: float,
                    momentum_coef: float, nesterov: bool, tails=None) -> None:
    """`outer_step` over T separate tensors per model (e.g. `list(model.parameters())` of
    models loaded on the GPU) in ONE launch, without packing: thetas[t], workers[k][t],
    momenta[t] (theta's dtype, required when momentum_coef != 0), all updated in place.
    tails: (bits, byte offsets) from torchcompat.torch_cpu_tail_bits_per_tensor — the reference
    host's bf16 scalar tails per tensor (edt_outer_step_list_tail; bf16 master only)."""
    lib = L.lib()
    T, K = len(thetas), len(workers)
    if K == 0:
        raise L.EdtError("no workers")
    if K > L.EDT_MAX_WORKERS:
        raise L.EdtError(f"tensor-list step takes at most {L.EDT_MAX_WORKERS} workers")
    if any(len(w) != T for w in workers):
        raise L.EdtError("every worker needs one tensor per parameter")
    if momentum_coef != 0 and momenta is None:
        raise L.EdtError("momentum tensors are required when momentum != 0")
    if momenta is not None and len(momenta) != T:
        raise L.EdtError("one momentum tensor per parameter")
    if T == 0:
        return
    # one comprehension per property over all T x (K + 2) tensors (the drop-in path sees
    # model.parameters() lists: hundreds of tensors per model, so per-tensor Python matters)
    flat_w = [t for w in workers for t in w]
    every = thetas + flat_w + (list(momenta) if momenta is not None else [])
    if not all([t.is_cuda for t in every]):
        raise L.EdtError("outer-loop sync operands must be device-resident (HBM) tensors")
    if not all([t.is_contiguous() for t in every]):
        raise L.EdtError("outer-loop sync operands must be contiguous")
    if len({t.get_device() for t in every}) != 1:
        raise L.EdtError("operands on different devices")
    gdt, wdt = thetas[0].dtype, workers[0][0].dtype
    if {t.dtype for t in thetas} != {gdt}:
        raise L.EdtError("all parameters of the base model must share one dtype")
    if {t.dtype for t in flat_w} != {wdt}:
        raise L.EdtError("every worker tensor must share the workers' dtype")
    numels = [t.numel() for t in thetas]
    for k, w in enumerate(workers):
        if [t.numel() for t in w] != numels:
            bad = next(t for t in range(T) if w[t].numel() != numels[t])
            raise L.EdtError(f"worker tensor {bad} does not match the base parameter")
    if momenta is not None:
        if [t.numel() for t in momenta] != numels or {t.dtype for t in momenta} != {gdt}:
            raise L.EdtError("momentum tensors must match the parameters' sizes and dtype")
    numel = (ctypes.c_uint64 * T)(*numels)
    nbytes = lib.edt_outer_list_workspace_bytes(T, K)
    ws = torch.empty(nbytes, dtype=torch.uint8, device=thetas[0].device)
    P_ = ctypes.c_void_p
    th_arr = (P_ * T)(*[t.data_ptr() for t in thetas])
    w_arr = (P_ * len(flat_w))(*[t.data_ptr() for t in flat_w])
    m_arr = (P_ * T)(*[t.data_ptr() for t in momenta]) if momenta is not None else None
    if tails is None:
        L.check(lib.edt_outer_step_list(th_arr, L.dtype_code(gdt), w_arr, L.dtype_code(wdt), K, m_arr,
                                        int(has_momentum), numel, T, float(lr), float(momentum_coef), int(nesterov),
                                        L.ptr(ws), nbytes, L.stream_ptr(thetas[0].device)), "edt_outer_step_list")
        return
    bits, offs = tails
    if gdt != torch.bfloat16:
        raise L.EdtError("scalar-tail bits apply to a bf16 master only")
    if len(offs) != T or not bits.is_cuda or bits.dtype != torch.uint8 or bits.device != thetas[0].device:
        raise L.EdtError("tails: a uint8 device mask and one byte offset per tensor")
    if any(o + (n + 7) // 8 > bits.numel() for o, n in zip(offs, numels)):
        raise L.EdtError("tails: the mask does not cover every tensor")
    toff = (ctypes.c_uint64 * T)(*[int(o) for o in offs])
    L.check(lib.edt_outer_step_list_tail(th_arr, L.dtype_code(gdt), w_arr, L.dtype_code(wdt), K, m_arr,
                                         int(has_momentum), numel, T, float(lr), float(momentum_coef), int(nesterov),
                                         L.ptr(bits), toff, L.ptr(ws), nbytes, L.stream_ptr(thetas[0].device)),
            "edt_outer_step_list_tail")


def delta_partial(theta: torch.Tensor, workers: list[torch.Tensor], k_total: int,
                  acc: torch.Tensor, accumulate: bool = False) -> None:
    """acc (fp32) (+)= sum over the local workers of round((theta_k - theta) / k_total)."""
    lib = L.lib()
    L.require_device(theta, acc, *workers)
    if acc.dtype != torch.float32 or acc.numel() != theta.numel():
        raise L.EdtError("acc must be a float32 buffer of theta's size")
    L.check(lib.edt_delta_partial(L.ptr(theta), L.dtype_code(theta), L.ptr_array(workers),
                                  L.dtype_code(workers[0]), len(workers), int(k_total),
                                  theta.numel(), L.ptr(acc), int(accumulate),
                                  L.stream_ptr(theta.device)), "edt_delta_partial")


def sgd_apply(theta: torch.Tensor, acc: torch.Tensor, momentum: torch.Tensor | None,
              has_momentum: bool, lr: float, momentum_coef: float, nesterov: bool) -> None:
    """grad = -round(acc); torch.optim.SGD step on theta (shard) in place."""
    lib = L.lib()
    L.require_device(theta, acc, momentum)
    if acc.dtype != torch.float32 or acc.numel() != theta.numel():
        raise L.EdtError("acc must be a float32 buffer of theta's size")
    L.check(lib.edt_sgd_apply(L.ptr(theta), L.dtype_code(theta), L.ptr(acc), L.ptr(momentum),
                              int(has_momentum), theta.numel(), float(lr), float(momentum_coef),
                              int(nesterov), L.stream_ptr(theta.device)), "edt_sgd_apply")


def sgd_apply_sum(theta: torch.Tensor, accs: list[torch.Tensor], momentum: torch.Tensor | None,
                  has_momentum: bool, lr: float, momentum_coef: float, nesterov: bool) -> None:
    """grad = -round(((acc_0 + acc_1) + ...)) in that order (fp32), then the SGD step on theta
    (edt_sgd_apply_sum: the reduce_ordered schedule's per-shard step)."""
    lib = L.lib()
    L.require_device(theta, momentum, *accs)
    if not accs or any(a.dtype != torch.float32 or a.numel() != theta.numel() for a in accs):
        raise L.EdtError("accs: fp32 buffers of theta's size")
    L.check(lib.edt_sgd_apply_sum(L.ptr(theta), L.dtype_code(theta), L.ptr_array(accs), len(accs), L.ptr(momentum),
                                  int(has_momentum), theta.numel(), float(lr), float(momentum_coef), int(nesterov),
                                  L.stream_ptr(theta.device)), "edt_sgd_apply_sum")


def pair_merge(b1: torch.Tensor, b2: torch.Tensor | None, m1: torch.Tensor, m2: torch.Tensor,
               out: torch.Tensor, momentum: torch.Tensor | None, has_momentum: bool, lr: float,
               momentum_coef: float, nesterov: bool, momentum_in: torch.Tensor | None = None,
               tail_bits: torch.Tensor | None = None) -> None:
    """EDT child = SGD step of lerp(.5, b1, b2) towards m1, m2 (EDT_LM/train/crossover.py:150-230).
    b2 None: b1 is the already merged base (dtype of `out`). momentum is updated in place, or,
    with `momentum_in` (the donor parent's buffer, left intact), written fresh
    (edt_pair_merge_to)."""
    lib = L.lib()
    L.require_device(b1, b2, m1, m2, out, momentum, momentum_in)
    n = out.numel()
    if any(t is not None and t.numel() != n for t in (b1, b2, m1, m2, momentum, momentum_in)):
        raise L.EdtError("pair-merge buffers must all have the same size")
    # the kernel reads b1/b2/m2 as m1's dtype (b1 as out's when b2 is None) and both momenta as
    # out's dtype: a mismatch would reinterpret raw bytes
    if b2 is not None:
        if not (b1.dtype == b2.dtype == m1.dtype == m2.dtype):
            raise L.EdtError("b1, b2, m1 and m2 must share one dtype")
    elif b1.dtype != out.dtype or m1.dtype != m2.dtype:
        raise L.EdtError("with b2=None, b1 (the merged base) must have out's dtype and m1, m2 one dtype")
    if any(t is not None and t.dtype != out.dtype for t in (momentum, momentum_in)):
        raise L.EdtError("momentum buffers must have out's dtype")
    mom_in = momentum if momentum_in is None else momentum_in
    if tail_bits is not None:
        L.require_device(tail_bits)
        if tail_bits.dtype != torch.uint8 or tail_bits.numel() * 8 < n:
            raise L.EdtError("tail_bits: uint8 with one bit per element")
    L.check(lib.edt_pair_merge_tail(L.ptr(b1), L.ptr(b2), L.ptr(m1), L.ptr(m2), L.dtype_code(m1),
                                    L.ptr(out), L.dtype_code(out), L.ptr(mom_in), L.ptr(momentum),
                                    int(has_momentum), n, float(lr), float(momentum_coef), int(nesterov),
                                    L.ptr(tail_bits), L.stream_ptr(out.device)), "edt_pair_merge_tail")


def lerp(t: float, v0: torch.Tensor, v1: torch.Tensor, out: torch.Tensor | None = None,
         compute_dtype: torch.dtype | None = None) -> torch.Tensor:
    """(1-t)*v0 + t*v1 with the rounding of three torch ops in compute_dtype (default: v0's)."""
    lib = L.lib()
    cdt = compute_dtype or v0.dtype
    if out is None:
        out = torch.empty_like(v0, dtype=cdt)
    L.require_device(v0, v1, out)
    if v1.dtype != v0.dtype or v1.numel() != v0.numel() or out.numel() != v0.numel():
        raise L.EdtError("lerp operands must match")
    L.check(lib.edt_lerp(L.ptr(v0), L.ptr(v1), L.dtype_code(v0), L.ptr(out), L.dtype_code(out),
                         L.dtype_code(cdt), v0.numel(), float(t), L.stream_ptr(v0.device)), "edt_lerp")
    return out


# ------------------------------------------------------------------------------------------
# SLERP over a multi-tensor arena

_TLS = threading.local()             # per host thread: {(device, stream): float64 buffer}


def _thread_slot(owner: dict, name: str) -> dict:
    """owner[name]'s dict for the calling host thread (created empty), held weakly by the thread
    object: a plan's per-thread workspaces are released with the thread that made them."""
    import weakref
    per = owner.get(name)
    if per is None:
        per = owner.setdefault(name, weakref.WeakKeyDictionary())
    th = threading.current_thread()
    slot = per.get(th)
    if slot is None:
        slot = per.setdefault(th, {})
    return slot


def _scratch(device: torch.device, ndoubles: int) -> torch.Tensor:
    """float64 device workspace of `ndoubles` (a view) from one growing buffer per (device, stream)
    of the calling host thread. The chunk-sum passes' rows and row scratch are only live inside one
    call, so every plan shares one buffer instead of each cached plan holding its own (7B body:
    107,893 chunks x 387 doubles = 334 MB for a pair merge; the population speculative form 3,096
    doubles per chunk at 8 children = 2.7 GB). Calls issued by one thread on one
    stream run in order, so a later call overwrites the rows only after the earlier call's kernels
    are done; threads issuing onto one stream (virtual ranks) interleave their launches, hence a
    buffer per thread (released with the thread)."""
    pools = getattr(_TLS, "pools", None)
    if pools is None:
        pools = _TLS.pools = {}
    dev = torch.device(device)
    idx = dev.index if dev.index is not None else torch.cuda.current_device()
    key = (idx, torch.cuda.current_stream(dev).cuda_stream)
    buf = pools.get(key)
    n = max(1, int(ndoubles))
    if buf is None or buf.numel() < n:
        pools.pop(key, None)
        buf = pools[key] = torch.empty(n, dtype=torch.float64, device=dev)
    return buf[:n]


def release_scratch() -> None:
    """Drop this thread's pooled SLERP workspaces (bench.py frees them between workloads)."""
    _TLS.pools = {}


@dataclass
class SlerpPlan:
    """Chunk table for a segment layout, resident on the device (built once per layout)."""
    seg_offsets: list[int]
    chunks: torch.Tensor          # int64 [nchunks, 3] = start, length, segment
    seg_first: torch.Tensor       # int32 [nseg + 1]
    nchunks: int
    relative: bool = False        # chunk starts relative to their segment (tensor-list form)
    chunks_host: object = None    # numpy int64 [nchunks, 3]: the same table on the host
    chunk_elems: int = 1 << 16

    @property
    def nseg(self) -> int:
        return len(self.seg_offsets) - 1

    def ws(self, name: str, n: int, dtype: torch.dtype) -> torch.Tensor:
        """The device workspace `name` on this plan of the calling host thread and its current
        stream (>= n elements, grown on demand; a view of n): plans are shared (merge._plan_for, the
        population planners), host threads (virtual ranks) may merge over one plan at the same time,
        and one thread may issue merges over one plan on two streams without syncing between them —
        each (thread, stream) reads back its own coefficients and dots, as _scratch keys its rows."""
        per = _thread_slot(self.__dict__, "_ws_by_thread")
        n = max(1, int(n))
        dev = self.chunks.device
        key = (name, torch.cuda.current_stream(dev).cuda_stream if dev.type == "cuda" else 0)
        buf = per.get(key)
        if buf is None or buf.numel() < n or buf.dtype != dtype:
            buf = per[key] = torch.empty(n, dtype=dtype, device=dev)
        return buf[:n]

    @property
    def coef(self) -> torch.Tensor:
        """float32 [nseg, 2]: the last merge's per-segment coefficients (this host thread's)."""
        return self.ws("coef", 2 * max(1, self.nseg), torch.float32).view(max(1, self.nseg), 2)

    @property
    def dots(self) -> torch.Tensor:
        """float32 [nseg]: the last merge's per-segment dots (this host thread's)."""
        return self.ws("dots", self.nseg, torch.float32)

    @property
    def partial(self) -> torch.Tensor:
        """The pair passes' workspace: chunk rows [nchunks, 3] first, then the row scratch and the
        any-redo word (edt_slerp_sums_doubles(3, nchunks) doubles, pooled per stream)."""
        return _scratch(self.chunks.device, L.load_library().edt_slerp_sums_doubles(3, self.nchunks))

    @property
    def seg_numel(self):
        """numpy int64 [nseg]: the segments' sizes (cached)."""
        got = self.__dict__.get("_seg_numel")
        if got is None:
            import numpy as np
            got = self.__dict__["_seg_numel"] = np.diff(np.asarray(self.seg_offsets, dtype=np.int64))
        return got


def make_slerp_plan(seg_offsets: list[int], device: torch.device,
                    chunk_elems: int = 1 << 16, relative: bool = False) -> SlerpPlan:
    """relative=True: chunk starts are offsets inside their segment, for `slerp_list` over
    separate tensors (one segment per tensor)."""
    lib = L.load_library()
    nseg = len(seg_offsets) - 1
    offs = (ctypes.c_uint64 * max(1, nseg + 1))(*seg_offsets)
    first = (ctypes.c_int32 * (nseg + 1))()
    need = lib.edt_slerp_make_chunks(offs, nseg, chunk_elems, None, 0, first)
    nchunks = -need - 1 if need < 0 else need
    desc = (ctypes.c_uint64 * max(1, 3 * nchunks))()
    got = lib.edt_slerp_make_chunks(offs, nseg, chunk_elems, desc, nchunks, first)
    if got != nchunks:
        L.check(-1, "edt_slerp_make_chunks")
    import numpy as np
    host = np.ctypeslib.as_array(desc).astype(np.int64)[:3 * nchunks].copy().reshape(-1, 3)
    if relative and nchunks:
        host[:, 0] -= np.asarray(seg_offsets, dtype=np.int64)[host[:, 2]]
    chunks = torch.from_numpy(host).to(device)
    seg_first = torch.tensor(list(first), dtype=torch.int32).to(device)
    return SlerpPlan(list(seg_offsets), chunks, seg_first, nchunks, relative, host, int(chunk_elems))


# The host the reference-dot mode reproduces: the one tests/golden/ was recorded on
# (tests/golden/refdot_host.json, tests/golden/gen_refdot_host.py).
REFDOT_DOT_KERNEL = "openblas 0.3.29 SkylakeX"
REFDOT_COEF_DISPATCH = (("arccos", "AVX512_SKX"), ("sin", "AVX512_SKX"))
_REFDOT_CHECKED: set = set()


class RefDotHostWarning(UserWarning):
    """The running host's numpy dispatch or BLAS core differs from the reference-dot mode's."""


_HOST_DISPATCH = None


def host_dispatch() -> dict:
    """The running host's side of the reference-dot mode (cached): numpy's version, the SIMD target
    its float32 arccos / sin loops dispatch to (numpy.lib.introspect.opt_func_info; the
    NPY_DISABLE_CPU_FEATURES / CPU features of this process), and numpy's BLAS core as
    "<internal api> <version> <architecture>" (threadpoolctl; None when not importable)."""
    global _HOST_DISPATCH
    if _HOST_DISPATCH is None:
        import numpy as np
        disp = {}
        try:                                    # numpy >= 2.0 only
            from numpy.lib import introspect
            for f in ("arccos", "sin"):
                info = introspect.opt_func_info(func_name=f"^{f}$", signature="float32").get(f, {})
                disp[f] = next(iter(info.values()), {}).get("current")
        except (ImportError, AttributeError):
            disp = {"arccos": "unknown", "sin": "unknown"}      # host_mismatch reports it (strict: raises)
        blas, threads = None, None
        try:
            from threadpoolctl import threadpool_info
            for lib in threadpool_info():
                if lib.get("user_api") == "blas" and "numpy" in str(lib.get("filepath", "")):
                    blas = f"{lib.get('internal_api')} {lib.get('version')} {lib.get('architecture')}"
                    threads = lib.get("num_threads")
                    break
        except ImportError:
            pass
        _HOST_DISPATCH = {"numpy": np.__version__, "coef_dispatch": disp, "blas": blas, "blas_threads": threads}
    return _HOST_DISPATCH


@dataclass(frozen=True)
class RefDot:
    """Reference-dot mode (include/edt_sync.h, edt_slerp_refdot): segments whose fp64 dot lies
    within `band` of DOT_THRESHOLD (band < 0: every segment) take the reference's own fp32 dot —
    BLAS sdot norms + numpy's pairwise sum, restated bit for bit for the reference host's numpy /
    OpenBLAS (`threads` = OpenBLAS's thread count for sdot there; 1 on the pinned host) — and then
    EVERY segment's branch and coefficients are formed from its dot exactly as
    EDT_RL/crossover.py:31-43 forms them: numpy float32 arccos / sin / divisions on the host
    (reference_coefficients). With band < 0 the merge is the reference's, bit for bit. Without it
    (the default) the kernels decide from their fp64 dot, the accurate one, and form the
    coefficients on the device. Every SLERP form takes it (arena, tensor list,
    population, sharded population); it synchronises the host once per merge.

    The mode reproduces ONE host: `dot_kernel` is the BLAS dot restated on the device and
    `coef_dispatch` the SIMD targets numpy's float32 arccos / sin loops dispatch to there (the
    targets compute different bits: AVX512_SKX's SVML arccos and the baseline libm one differ on
    ~36 % of 400k float32 dots, sin 30 %: scripts/numpy_dispatch_probe.py). The defaults are the
    host tests/golden/ was recorded on (tests/golden/refdot_host.json). At first use the running
    host (host_dispatch()) is compared
    with them: a difference warns (RefDotHostWarning) — or raises with strict=True — since the
    coefficients would then not be the reference's bits on this host."""
    threads: int = 1
    band: float = -1.0
    dot_kernel: str = REFDOT_DOT_KERNEL
    coef_dispatch: tuple = REFDOT_COEF_DISPATCH
    strict: bool = False

    def host_mismatch(self) -> list[str]:
        """What differs between the running host and the host this mode reproduces ([] = none).
        A dispatch numpy cannot report (numpy < 2: no numpy.lib.introspect) counts as a difference.
        numpy's BLAS pool size is not compared: OpenBLAS decides per call how many threads sdot
        uses (the golden host reported 8 and its dots are reproduced with threads = 1), so the pool
        does not say it; `threads` is the parameter that does."""
        host = host_dispatch()
        out = [f"numpy float32 {f} dispatches to {host['coef_dispatch'].get(f)}, the modelled host's to {want}"
               for f, want in self.coef_dispatch if host["coef_dispatch"].get(f) != want]
        blas = host.get("blas")
        if blas is not None and blas != self.dot_kernel:
            out.append(f"numpy's BLAS dot is {blas}, the mode restates {self.dot_kernel}")
        return out

    def describe(self) -> dict:
        """The modelled host, the running one and whether they agree (for logs and bench lines)."""
        return {"dot_kernel": self.dot_kernel, "threads": self.threads, "coef_dispatch": dict(self.coef_dispatch),
                "host": host_dispatch(), "mismatch": self.host_mismatch()}

    def check_host(self) -> None:
        """Warn (strict: raise EdtError) once per setting when the running host differs."""
        key = (self.dot_kernel, self.coef_dispatch, self.strict)
        if key in _REFDOT_CHECKED:
            return
        bad = self.host_mismatch()
        if bad and self.strict:
            raise L.EdtError("reference-dot mode: this host is not the one it reproduces: " + "; ".join(bad))
        _REFDOT_CHECKED.add(key)
        if bad:
            import warnings
            warnings.warn("reference-dot mode: this host differs from the modelled one, the coefficients may not "
                          "be the reference's bits here: " + "; ".join(bad), RefDotHostWarning, stacklevel=3)


def reference_coefficients(dots, t, dot_threshold: float = 0.9995):
    """The reference's branch and (c0, c1) per segment (EDT_RL/crossover.py:31-43,
    EDT_EVOMERGE/train/crossover.py:34-46) from fp32 dots, evaluated the way the reference does:
    numpy float32 scalars (NEP 50: the python-float t and 1 - t enter as float32) — arccos, the
    product th0 * t, sin, two divisions — or, where |dot| > DOT_THRESHOLD, the lerp weights
    (1 - t, t). numpy's float32 arccos / sin are the reference's own dependency (SVML / numpy's SIMD
    loops on an AVX-512 host): no device restatement of them is bit-exact. dots: float32 [..., nseg];
    t: float64 [nseg]. Returns float32 [..., nseg, 2]."""
    import numpy as np
    d = np.asarray(dots, dtype=np.float32)
    tt = np.broadcast_to(np.asarray(t, dtype=np.float64), d.shape)
    tf = tt.astype(np.float32)
    with np.errstate(invalid="ignore", divide="ignore", over="ignore"):
        th0 = np.arccos(d)
        th_t = th0 * tf
        s0 = np.sin(th0 - th_t) / np.sin(th0)
        s1 = np.sin(th_t) / np.sin(th0)
    lerp = np.abs(d) > np.float32(dot_threshold)
    out = np.empty(d.shape + (2,), dtype=np.float32)
    out[..., 0] = np.where(lerp, (1.0 - tt).astype(np.float32), s0)
    out[..., 1] = np.where(lerp, tf, s1)
    return out


def _refdot_ws(plan: SlerpPlan, ref: RefDot, dev) -> torch.Tensor:
    lib = L.lib()
    need = int(lib.edt_slerp_refdot_workspace_bytes(plan.nseg, plan.nchunks, plan.chunk_elems, int(ref.threads)))
    if need == 0:
        raise L.EdtError(f"reference-dot mode needs chunks of a multiple of 8192 elements (plan: {plan.chunk_elems})")
    return plan.ws("refdot", (need + 7) // 8, torch.float64)


def _ref_dots(plan: SlerpPlan, dots: torch.Tensor, ref: RefDot, in_dt: int, dot_threshold: float, eps: float,
              v0: torch.Tensor | None = None, v1: torch.Tensor | None = None, table: torch.Tensor | None = None):
    """Flag the segments of `dots` (fp32 device [nseg]) within ref.band of the threshold and
    recompute their dot the reference's way over (v0, v1) arenas or a tensor-list table. Returns the
    (flag int32, value float32) device tensors; nothing is synchronised."""
    lib = L.lib()
    ref.check_host()
    dev, st = dots.device, L.stream_ptr(dots.device)
    ws = _refdot_ws(plan, ref, dev)
    flag = torch.empty(max(1, plan.nseg), dtype=torch.int32, device=dev)
    val = torch.empty(max(1, plan.nseg), dtype=torch.float32, device=dev)
    L.check(lib.edt_slerp_refdot_flags(L.ptr(dots), plan.nseg, float(dot_threshold), float(ref.band), L.ptr(flag), st),
            "edt_slerp_refdot_flags")
    if table is None:
        L.check(lib.edt_slerp_refdot(L.ptr(v0), L.ptr(v1), in_dt, L.ptr(plan.chunks), plan.nchunks,
                                     L.ptr(plan.seg_first), plan.nseg, plan.chunk_elems, L.ptr(flag),
                                     int(ref.threads), float(eps), L.ptr(val), L.ptr(ws), ws.numel() * 8, st),
                "edt_slerp_refdot")
    else:
        L.check(lib.edt_slerp_refdot_table(L.ptr(table), in_dt, L.ptr(plan.chunks), plan.nchunks,
                                           L.ptr(plan.seg_first), plan.nseg, plan.chunk_elems, L.ptr(flag),
                                           int(ref.threads), float(eps), L.ptr(val), L.ptr(ws), ws.numel() * 8, st),
                "edt_slerp_refdot_table")
    return flag, val


def _reference_finish(dots: torch.Tensor, flag: torch.Tensor, val: torch.Tensor, t: torch.Tensor, nseg: int,
                      dot_threshold: float, coef_used: torch.Tensor | None = None):
    """Host part of the reference-dot mode (one synchronisation): the final fp32 dots (the
    reference's where flagged), the reference's coefficients from them, and — given the
    coefficients a pass already blended with (`coef_used`, [.., nseg, 2]) — the segments whose
    coefficients changed. dots / flag / val: [..., nseg] device tensors. Returns (dots, coef,
    changed) as device tensors shaped like the inputs (changed: int32 or None)."""
    import numpy as np
    shp = dots.shape
    d = dots.reshape(-1, dots.shape[-1])[:, :nseg].cpu().numpy()
    f = flag.reshape(-1, flag.shape[-1])[:, :nseg].cpu().numpy()
    v = val.reshape(-1, val.shape[-1])[:, :nseg].cpu().numpy()
    th = t[:nseg].cpu().numpy()
    final = np.where(f != 0, v, d).astype(np.float32)
    coef = reference_coefficients(final, th, dot_threshold)
    dev = dots.device
    dots_out = torch.from_numpy(final).to(dev).reshape(shp[:-1] + (nseg,))
    coef_out = torch.from_numpy(coef).to(dev).reshape(shp[:-1] + (nseg, 2))
    changed = None
    if coef_used is not None:
        used = coef_used.reshape(-1, coef_used.shape[-2], 2)[:, :nseg].cpu().numpy()
        diff = (used.view(np.int32) != coef.view(np.int32)).any(axis=-1).astype(np.int32)
        changed = torch.from_numpy(diff).to(dev).reshape(shp[:-1] + (nseg,))
    return dots_out, coef_out, changed


def _dots_state(plan) -> dict:
    """The calling host thread's record of its previous merges' dots on this plan."""
    return _thread_slot(plan.__dict__, "_dots_by_thread")


def _record_dots(plan: SlerpPlan, dots: torch.Tensor, attr: str) -> None:
    """After a merge: the dots go to pinned host memory by an async copy on the merge's stream, with
    an event, so the next call (on this host thread) can judge its form without synchronising the
    device."""
    st = _dots_state(plan)
    host = st.get(attr + "_host")
    if host is None or host.shape != dots.shape:
        host = st[attr + "_host"] = torch.empty(dots.shape, dtype=dots.dtype, pin_memory=True)
    host.copy_(dots, non_blocking=True)
    ev = torch.cuda.Event()
    ev.record(torch.cuda.current_stream(dots.device))
    st[attr + "_event"] = ev


def _host_dots(plan: SlerpPlan, attr: str, wait: bool):
    """The previous merge's dots on the host (numpy), or None while its copy is still in flight
    (wait=False: never blocks; wait=True: waits for that copy only)."""
    st = _dots_state(plan)
    ev = st.get(attr + "_event")
    if ev is None:
        return None
    if wait:
        ev.synchronize()
    elif not ev.query():
        return None
    return st[attr + "_host"].numpy()


def _speculation_pays(plan: SlerpPlan, in_bytes: int, out_bytes: int, wait: bool = True) -> bool:
    """Whether the speculative form is cheaper for the next merge on this plan, judged from the
    dots the previous merge on it produced (both forms write them): with a fraction f of the
    elements in SLERP-branch segments it moves (1 + f)(2 b_in + b_out) bytes per element against
    4 b_in + b_out. No previous merge: speculate (EDT parents share a lineage). wait=False (what
    slerp_arena uses): when the previous merge's dots have not reached the host yet — calls issued
    back to back — the previous decision stands, so deciding never synchronises the device."""
    if getattr(plan, "_last_thr", None) is None:
        return True
    import numpy as np
    dots = _host_dots(plan, "_dots", wait)
    if dots is None:
        return getattr(plan, "_last_speculate", True)
    dots = dots[:plan.nseg]
    sizes = plan.seg_numel
    total = max(1, int(plan.seg_offsets[-1]))
    f = float(sizes[np.abs(dots) <= plan._last_thr].sum()) / total
    return (1 + f) * (2 * in_bytes + out_bytes) < 4 * in_bytes + out_bytes


def _overlap(a: torch.Tensor, b: torch.Tensor) -> bool:
    a0, b0 = a.data_ptr(), b.data_ptr()
    return a0 < b0 + b.numel() * b.element_size() and b0 < a0 + a.numel() * a.element_size()


def _pair_ref_merge(plan: SlerpPlan, in_dt: int, out_dt: int, t: torch.Tensor, dot_threshold: float, eps: float,
                    ref: RefDot, speculate: bool, arena=None, table=None, n: int = 0) -> None:
    """The reference-dot mode of one pair (flat arenas (v0, v1, out) or a tensor-list table):
      speculate=True   the speculative merge as usual (every segment's output = the blend with the
                       device's coefficients), then the reference's dots and coefficients, and a
                       re-blend of exactly the segments whose coefficients changed;
      speculate=False  stats -> device coefficients (their dots flag the band) -> the reference's
                       dots and coefficients -> one blend (an output may alias a parent).
    Either way every segment ends as the blend with the reference's coefficients: bit-identical
    across forms and layouts."""
    lib = L.lib()
    dev = t.device
    st = L.stream_ptr(dev)
    part = plan.partial
    if arena is not None:
        v0, v1, out = arena
    if speculate:
        redo = torch.empty(max(1, plan.nseg), dtype=torch.int32, device=dev)
        if arena is not None:
            L.check(lib.edt_slerp_merge_speculative(
                L.ptr(v0), L.ptr(v1), in_dt, L.ptr(out), out_dt, L.ptr(plan.chunks), plan.nchunks,
                L.ptr(plan.seg_first), plan.nseg, L.ptr(t), float(dot_threshold), float(eps), L.ptr(part),
                L.ptr(plan.coef), L.ptr(plan.dots), L.ptr(redo), n, st), "edt_slerp_merge_speculative")
        else:
            L.check(lib.edt_slerp_merge_table_speculative(
                L.ptr(table), in_dt, out_dt, L.ptr(plan.chunks), plan.nchunks, L.ptr(plan.seg_first), plan.nseg,
                L.ptr(t), float(dot_threshold), float(eps), L.ptr(part), L.ptr(plan.coef), L.ptr(plan.dots),
                L.ptr(redo), st), "edt_slerp_merge_table_speculative")
    else:
        if arena is not None:
            L.check(lib.edt_slerp_stats(L.ptr(v0), L.ptr(v1), in_dt, L.ptr(plan.chunks), plan.nchunks, L.ptr(part),
                                        st), "edt_slerp_stats")
        else:
            L.check(lib.edt_slerp_stats_table(L.ptr(table), in_dt, L.ptr(plan.chunks), plan.nchunks, L.ptr(part), st),
                    "edt_slerp_stats_table")
        L.check(lib.edt_slerp_coef(L.ptr(part), L.ptr(plan.seg_first), plan.nseg, L.ptr(t), float(dot_threshold),
                                   float(eps), L.ptr(plan.coef), L.ptr(plan.dots), st), "edt_slerp_coef")
    if arena is not None:
        flag, val = _ref_dots(plan, plan.dots, ref, in_dt, dot_threshold, eps, v0=v0, v1=v1)
    else:
        flag, val = _ref_dots(plan, plan.dots, ref, in_dt, dot_threshold, eps, table=table)
    dots, coef, changed = _reference_finish(plan.dots, flag, val, t, plan.nseg, dot_threshold,
                                            plan.coef if speculate else None)
    plan.dots[:plan.nseg].copy_(dots)
    plan.coef[:plan.nseg].copy_(coef)
    if arena is not None:
        if speculate:
            L.check(lib.edt_slerp_blend_segments(L.ptr(v0), L.ptr(v1), in_dt, L.ptr(out), out_dt, L.ptr(plan.chunks),
                                                 plan.nchunks, L.ptr(plan.coef), L.ptr(changed), st),
                    "edt_slerp_blend_segments")
        else:
            L.check(lib.edt_slerp_blend(L.ptr(v0), L.ptr(v1), in_dt, L.ptr(out), out_dt, L.ptr(plan.chunks),
                                        plan.nchunks, L.ptr(plan.coef), st), "edt_slerp_blend")
    else:
        L.check(lib.edt_slerp_blend_table(L.ptr(table), in_dt, out_dt, L.ptr(plan.chunks), plan.nchunks,
                                          L.ptr(plan.coef), L.ptr(changed) if speculate else None, st),
                "edt_slerp_blend_table")


def slerp_arena(plan: SlerpPlan, v0: torch.Tensor, v1: torch.Tensor, out: torch.Tensor,
                t: torch.Tensor, dot_threshold: float = 0.9995, eps: float = 1e-8,
                speculate: bool | None = None, ref_dot: RefDot | None = None) -> None:
    """SLERP every segment of v0/v1 with its own t (float64 device tensor [nseg]) into out
    (EDT_RL/crossover.py:11-43): chunk sums, per-segment coefficients, blend (edt_slerp_merge).
    speculate: True = edt_slerp_merge_speculative (lerp-branch output written in the stats pass,
    only SLERP-branch segments blended again); False = the two-pass form; None = whichever the
    previous merge on this plan says is cheaper. Bit-identical results either way; an output
    that overlaps a parent always takes the two-pass form. ref_dot (RefDot): the reference-dot
    mode (the reference's dots and coefficients, bit for bit with band < 0), either form."""
    lib = L.lib()
    L.require_device(v0, v1, out, t)
    if v1.dtype != v0.dtype or v0.numel() != plan.seg_offsets[-1] or v1.numel() != v0.numel() \
            or out.numel() != v0.numel():
        raise L.EdtError("slerp arenas must match the plan's layout")
    if t.dtype != torch.float64 or t.numel() < plan.nseg:
        raise L.EdtError("t must be a float64 device tensor with one value per segment")
    if plan.relative:
        raise L.EdtError("a relative (tensor-list) plan drives slerp_list, not slerp_arena")
    if speculate is None:
        speculate = _speculation_pays(plan, v0.element_size(), out.element_size(), wait=False)
        plan._last_speculate = speculate
    if speculate and (_overlap(out, v0) or _overlap(out, v1)):
        speculate = False
    if ref_dot is not None:
        _pair_ref_merge(plan, L.dtype_code(v0), L.dtype_code(out), t, dot_threshold, eps, ref_dot, speculate,
                        arena=(v0, v1, out), n=v0.numel())
    elif speculate:
        redo = plan.ws("redo", plan.nseg, torch.int32)
        L.check(lib.edt_slerp_merge_speculative(
            L.ptr(v0), L.ptr(v1), L.dtype_code(v0), L.ptr(out), L.dtype_code(out), L.ptr(plan.chunks), plan.nchunks,
            L.ptr(plan.seg_first), plan.nseg, L.ptr(t), float(dot_threshold), float(eps), L.ptr(plan.partial),
            L.ptr(plan.coef), L.ptr(plan.dots), L.ptr(redo), v0.numel(), L.stream_ptr(v0.device)),
            "edt_slerp_merge_speculative")
    else:
        L.check(lib.edt_slerp_merge(L.ptr(v0), L.ptr(v1), L.dtype_code(v0), L.ptr(out), L.dtype_code(out),
                                    L.ptr(plan.chunks), plan.nchunks, L.ptr(plan.seg_first), plan.nseg, L.ptr(t),
                                    float(dot_threshold), float(eps), L.ptr(plan.partial), L.ptr(plan.coef),
                                    L.ptr(plan.dots), L.stream_ptr(v0.device)), "edt_slerp_merge")
    plan._last_thr = float(dot_threshold)
    _record_dots(plan, plan.dots[:max(1, plan.nseg)], "_dots")


def writes_safe(starts, nbytes) -> bool:
    """The tensor-list SLERP's write rule over byte spans laid out as (v0, v1, out) per segment
    (numpy int64 [3 nseg] each): out[i] may alias its own inputs exactly (the blend is element-wise,
    after every sum); any other overlap of an output with an input or another output is unsafe in
    either form. Identical spans are grouped; a group holding an output may hold only spans of that
    output's own segment; distinct groups that overlap are unsafe when either holds an output (a
    sorted sweep: running furthest end of every group / of the groups holding an output)."""
    import numpy as np
    st = np.asarray(starts, dtype=np.int64)
    nb = np.asarray(nbytes, dtype=np.int64)
    nseg = st.size // 3
    kind_out = np.tile(np.array([False, False, True]), nseg)
    owner = np.repeat(np.arange(nseg, dtype=np.int64), 3)
    keep = nb > 0
    st, en, kind_out, owner = st[keep], st[keep] + nb[keep], kind_out[keep], owner[keep]
    if st.size == 0:
        return True
    order = np.lexsort((en, st))
    st, en, kind_out, owner = st[order], en[order], kind_out[order], owner[order]
    new_group = np.ones(st.size, dtype=bool)
    new_group[1:] = (st[1:] != st[:-1]) | (en[1:] != en[:-1])
    gid = np.cumsum(new_group) - 1
    ng = int(gid[-1]) + 1
    outs_per = np.bincount(gid, weights=kind_out, minlength=ng)
    if (outs_per > 1).any():
        return False                                         # two outputs on one span
    out_owner = np.full(ng, -1, dtype=np.int64)
    out_owner[gid[kind_out]] = owner[kind_out]
    has_out = out_owner >= 0
    if (has_out[gid] & (owner != out_owner[gid])).any():
        return False                                         # an output on another segment's span
    gst, gen = st[new_group], en[new_group]
    prev_end = np.concatenate(([-1], np.maximum.accumulate(gen)[:-1]))
    prev_out_end = np.concatenate(([-1], np.maximum.accumulate(np.where(has_out, gen, -1))[:-1]))
    return not bool(np.any((has_out & (gst < prev_end)) | (gst < prev_out_end)))


_ELEM_SIZE = {torch.float32: 4, torch.bfloat16: 2, torch.float16: 2, torch.float64: 8}


def _stage_state(plan) -> dict:
    """The calling host thread's staging state on this plan: plans are shared (merge._plan_for),
    and host threads (virtual ranks) may bind on one plan at the same time."""
    st = _thread_slot(plan.__dict__, "_table_stage_state")
    if not st:
        st.update(stages=[None, None], events=[None, None], next=1)
    return st


def _table_stage(plan, n3: int) -> torch.Tensor:
    """One of the calling thread's two pinned staging buffers on this plan for a pointer-table image
    (>= n3 int64), in turn, once the upload from it two bindings ago has completed: the image is
    written there and goes up by an async copy (a pageable upload waits for its own staging, the
    largest host cost of a repeated binding); alternating buffers, a binding never waits for the
    previous one's copy, which may sit behind other work on the stream."""
    st = _stage_state(plan)
    k = st["next"] = 1 - st["next"]
    stage, ev = st["stages"][k], st["events"][k]
    if ev is not None:
        ev.synchronize()                         # the buffer may still be read by its copy
    if stage is None or stage.numel() < n3:
        stage = st["stages"][k] = torch.zeros(n3, dtype=torch.int64, pin_memory=torch.cuda.is_available())
    return stage


def _table_upload(plan, stage: torch.Tensor, n3: int, device) -> torch.Tensor:
    if device is not None and device.type == "cuda":
        table = torch.empty(n3, dtype=torch.int64, device=device)
        table.copy_(stage[:n3], non_blocking=True)
        ev = torch.cuda.Event()
        ev.record(torch.cuda.current_stream(device))
        st = _stage_state(plan)
        st["events"][st["next"]] = ev
        return table
    return stage[:n3].clone()


class SlerpListBinding:
    """A tensor-list SLERP bound to its tensors (EDT_EVOMERGE/train/crossover.py:104-146's state-dict
    tensors, merged where they lie): the per-tensor checks run once here and the validated
    {v0, v1, out} pointer table (edt_slerp_seg_table) is uploaded once, so `merge` costs no
    per-tensor host work. The tensors must stay where they are while the binding is used (it keeps
    references to them; rebinding a module's parameters elsewhere needs a new binding)."""

    def __init__(self, plan: SlerpPlan, v0s, v1s, outs, checked: bool = False):
        """checked=True (merge.slerp_tensors): the caller has verified devices, contiguity, sizes
        against the plan and the two dtypes; the per-tensor Python pass is skipped (alignment and
        the overlap rule are checked in C either way)."""
        import numpy as np
        lib = L.lib()
        T = len(v0s)
        if not plan.relative or T != plan.nseg or len(v1s) != T or len(outs) != T:
            raise L.EdtError("slerp_list needs a relative plan with one segment per tensor")
        in_dt, out_dt = (v0s[0].dtype, outs[0].dtype) if T else (torch.float32, torch.float32)
        keep = (list(v0s), list(v1s), list(outs))
        if checked and T:
            self.device = v0s[0].device
            p0, p1, po = (np.fromiter((x.data_ptr() for x in ts), dtype=np.uint64, count=T) for ts in keep)
        else:
            # one pass over the triples (what L.require_device and the size / dtype checks test)
            p0, p1, po, devs = [], [], [], set()
            for i, (x, y, o, n) in enumerate(zip(*keep, plan.seg_numel.tolist())):
                if not (x.is_cuda and y.is_cuda and o.is_cuda):
                    raise L.EdtError("outer-loop sync operands must be device-resident (HBM) tensors")
                if not (x.is_contiguous() and y.is_contiguous() and o.is_contiguous()):
                    raise L.EdtError("outer-loop sync operands must be contiguous")
                if x.numel() != n or y.numel() != n or o.numel() != n:
                    raise L.EdtError(f"tensor {i} does not match the plan's layout")
                if x.dtype != in_dt or y.dtype != in_dt or o.dtype != out_dt:
                    raise L.EdtError("slerp_list: one input dtype and one output dtype")
                devs.update((x.get_device(), y.get_device(), o.get_device()))
                p0.append(x.data_ptr())
                p1.append(y.data_ptr())
                po.append(o.data_ptr())
            if len(devs) > 1:
                raise L.EdtError(f"operands on different devices: {sorted(devs)}")
            self.device = v0s[0].device if T else None
            p0, p1, po = (np.array(p, dtype=np.uint64) for p in (p0, p1, po))
        self._bind(plan, p0, p1, po, in_dt, out_dt, keep)

    @classmethod
    def from_pointers(cls, plan: SlerpPlan, p0, p1, pout, in_dtype: torch.dtype, out_dtype: torch.dtype,
                      device: torch.device, keep) -> "SlerpListBinding":
        """A binding over raw device addresses (numpy uint64 [nseg] each: v0, v1, out of every
        segment, sizes = the plan's), for a caller that has checked devices, contiguity, dtypes and
        sizes itself (merge.slerp_into_module_: the children's addresses in a fresh buffer are known
        before any view of it exists). Alignment and the overlap rule are still checked in C.
        `keep`: whatever owns the memory (held as long as the binding)."""
        self = cls.__new__(cls)
        if not plan.relative or not (len(p0) == len(p1) == len(pout) == plan.nseg):
            raise L.EdtError("slerp_list needs a relative plan with one segment per tensor")
        self.device = device
        self._bind(plan, p0, p1, pout, in_dtype, out_dtype, keep)
        return self

    def _bind(self, plan, p0, p1, po, in_dt, out_dt, keep):
        import numpy as np
        lib, T = L.load_library(), plan.nseg       # host validation only; merge() insists on the device
        self.plan, self.in_dt, self.out_dt = plan, L.dtype_code(in_dt), L.dtype_code(out_dt)
        self.in_size, self.out_size = _ELEM_SIZE[in_dt], _ELEM_SIZE[out_dt]
        self._keep = keep
        arrs = [np.ascontiguousarray(a if T else np.zeros(1), dtype=np.uint64) for a in (p0, p1, po)]
        vp = ctypes.POINTER(ctypes.c_void_p)
        a0, a1, a2 = (a.ctypes.data_as(vp) for a in arrs)
        numel_arr = np.ascontiguousarray(plan.seg_numel, dtype=np.uint64)   # alive across both calls below
        numel = numel_arr.ctypes.data_as(ctypes.c_void_p) if T else None
        n3 = max(1, 3 * T)
        stage = _table_stage(plan, n3)
        hp = ctypes.c_void_p(stage.data_ptr())
        # every output apart from everything but its own parents (the two-pass form's rule, r5: in C)
        L.check(lib.edt_slerp_seg_table(a0, a1, a2, T, numel, self.in_dt, self.out_dt, 0, hp), "edt_slerp_seg_table")
        # outputs apart from every parent (a sorted-span check in C): the single-pass form is allowed
        self.apart = lib.edt_slerp_seg_table(a0, a1, a2, T, numel, self.in_dt, self.out_dt, 1, hp) == 0
        self.table = _table_upload(plan, stage, n3, self.device)

    @classmethod
    def from_checked(cls, plan: SlerpPlan, p0, p1, pout, in_dtype: torch.dtype, out_dtype: torch.dtype,
                     device: torch.device, keep) -> "SlerpListBinding":
        """from_pointers for addresses that were validated before and cannot have changed
        (merge._Bound's repeat: the parents' addresses are exactly those an earlier binding checked,
        with their memory held; the outputs are views of a fresh buffer at 16-byte aligned offsets,
        apart from every parent by construction). The table image is written without the C checks
        (every invariant they test holds by construction), into the plan's pinned staging buffer."""
        import numpy as np
        self = cls.__new__(cls)
        T = plan.nseg
        if not plan.relative or not (len(p0) == len(p1) == len(pout) == T):
            raise L.EdtError("slerp_list needs a relative plan with one segment per tensor")
        self.device, self.plan = device, plan
        self.in_dt, self.out_dt = L.dtype_code(in_dtype), L.dtype_code(out_dtype)
        self.in_size, self.out_size = _ELEM_SIZE[in_dtype], _ELEM_SIZE[out_dtype]
        self._keep, self.apart = keep, True
        n3 = max(1, 3 * T)
        stage = _table_stage(plan, n3)
        img = stage.numpy()[:3 * T].reshape(T, 3).view(np.uint64)
        img[:, 0], img[:, 1], img[:, 2] = p0, p1, pout
        self.table = _table_upload(plan, stage, n3, device)
        return self

    def merge(self, t: torch.Tensor, dot_threshold: float = 0.9995, eps: float = 1e-8,
              speculate: bool | None = None, ref_dot: RefDot | None = None) -> None:
        """slerp_list's merge over the bound tensors (same forms, same results)."""
        lib, plan = L.lib(), self.plan
        if t.dtype != torch.float64 or t.numel() < plan.nseg or t.device != self.device:
            raise L.EdtError("t must be a float64 tensor on the tensors' device with one value per segment")
        if speculate is None:
            speculate = _speculation_pays(plan, self.in_size, self.out_size, wait=False)
            plan._last_speculate = speculate
        speculate = bool(speculate and self.apart)
        st = L.stream_ptr(self.device)
        if ref_dot is not None:
            _pair_ref_merge(plan, self.in_dt, self.out_dt, t, dot_threshold, eps, ref_dot, speculate, table=self.table)
        elif speculate:
            redo = plan.ws("redo", plan.nseg, torch.int32)
            L.check(lib.edt_slerp_merge_table_speculative(
                L.ptr(self.table), self.in_dt, self.out_dt, L.ptr(plan.chunks), plan.nchunks, L.ptr(plan.seg_first),
                plan.nseg, L.ptr(t), float(dot_threshold), float(eps), L.ptr(plan.partial), L.ptr(plan.coef),
                L.ptr(plan.dots), L.ptr(redo), st), "edt_slerp_merge_table_speculative")
        else:
            L.check(lib.edt_slerp_merge_table(
                L.ptr(self.table), self.in_dt, self.out_dt, L.ptr(plan.chunks), plan.nchunks, L.ptr(plan.seg_first),
                plan.nseg, L.ptr(t), float(dot_threshold), float(eps), L.ptr(plan.partial), L.ptr(plan.coef),
                L.ptr(plan.dots), st), "edt_slerp_merge_table")
        plan._last_thr = float(dot_threshold)
        _record_dots(plan, plan.dots[:max(1, plan.nseg)], "_dots")


def bind_slerp_list(plan: SlerpPlan, v0s, v1s, outs) -> SlerpListBinding:
    """A SlerpListBinding: validate once, merge many times without per-tensor host work."""
    return SlerpListBinding(plan, v0s, v1s, outs)


def slerp_list(plan: SlerpPlan, v0s: list[torch.Tensor], v1s: list[torch.Tensor], outs: list[torch.Tensor],
               t: torch.Tensor, dot_threshold: float = 0.9995, eps: float = 1e-8,
               speculate: bool | None = None, ref_dot: RefDot | None = None) -> None:
    """`slerp_arena` over separate tensors (one segment each, e.g. two models' state-dict
    tensors), writing straight into `outs` (e.g. the target model's parameters): no packing.
    Every tensor must be contiguous and 16-byte aligned; plan = make_slerp_plan(...,
    relative=True) over the tensors' sizes. speculate as slerp_arena's: True = the single-pass
    form (lerp-branch outputs written in the sums pass, only SLERP-branch tensors blended again),
    False = the two-pass form, None = the cheaper by the previous merge's dots on this plan;
    outputs that overlap any parent (e.g. merged into the first parent's own tensors) always take
    the two-pass form. Bit-identical either way. ref_dot: the reference-dot mode, as slerp_arena's.
    Validates and uploads the tensors' pointer table on every call; a caller that merges the same
    tensors again holds a `bind_slerp_list` binding instead."""
    SlerpListBinding(plan, v0s, v1s, outs).merge(t, dot_threshold, eps, speculate, ref_dot)


def _population_ref(plan: SlerpPlan, members, pairs, outs, t, dots, coef_used, in_dt, out_dt, dot_threshold, eps,
                    ref: RefDot, blend_all: bool):
    """Reference-dot mode for every child of a population: per child the reference's dots over its
    two parents (flagged by that child's dots), the reference's coefficients, then either the
    blend of every child (blend_all: no output written yet) or per child the re-blend of the
    segments whose coefficients changed. Returns (dots, coef) [Q, nseg(, 2)]."""
    lib = L.lib()
    Q, dev = len(pairs), t.device
    st = L.stream_ptr(dev)
    flags, vals = [], []
    for q, (i, j) in enumerate(pairs):
        f, v = _ref_dots(plan, dots[q], ref, in_dt, dot_threshold, eps, v0=members[i], v1=members[j])
        flags.append(f)
        vals.append(v)
    fd, cd, changed = _reference_finish(dots[:Q], torch.stack(flags), torch.stack(vals), t, plan.nseg,
                                        dot_threshold, None if blend_all else coef_used[:Q])
    coef = torch.empty((max(1, Q), max(1, plan.nseg), 2), dtype=torch.float32, device=dev)
    coef[:Q, :plan.nseg].copy_(cd)
    if blend_all:
        for q0 in range(0, Q, 16):
            q1 = min(Q, q0 + 16)
            slerp_blend_children(members, pairs[q0:q1], outs[q0:q1], plan.chunks, plan.nchunks,
                                 coef[q0:q1].contiguous(), max(1, plan.nseg))
    else:
        for q, (i, j) in enumerate(pairs):
            L.check(lib.edt_slerp_blend_segments(L.ptr(members[i]), L.ptr(members[j]), in_dt, L.ptr(outs[q]), out_dt,
                                                 L.ptr(plan.chunks), plan.nchunks, L.ptr(coef[q]), L.ptr(changed[q]),
                                                 st), "edt_slerp_blend_segments")
    return fd, coef


def slerp_refdot(v0: torch.Tensor, v1: torch.Tensor, chunks: torch.Tensor, seg_first: torch.Tensor, nseg: int,
                 chunk_elems: int, flag: torch.Tensor, ref: RefDot, eps: float = 1e-8) -> torch.Tensor:
    """The reference's fp32 dot (edt_slerp_refdot) of the flagged segments (flag: int32 device
    [nseg]) of a chunk table over two flat buffers (chunk starts relative to them; seg_first: int32
    device [nseg + 1] indexing the table's rows). float32 [nseg] device; unflagged entries are
    undefined. The sharded population's per-rank pass (distributed.ShardedPopulationCrossover)."""
    lib = L.lib()
    dev = L.require_device(v0, v1, chunks, seg_first, flag)
    nchunks = int(chunks.shape[0]) if chunks.dim() == 2 else int(chunks.numel()) // 3
    need = int(lib.edt_slerp_refdot_workspace_bytes(nseg, nchunks, int(chunk_elems), int(ref.threads)))
    if need == 0:
        raise L.EdtError(f"reference-dot mode needs chunks of a multiple of 8192 elements (got {chunk_elems})")
    ws = torch.empty((need + 7) // 8, dtype=torch.float64, device=dev)
    val = torch.empty(max(1, nseg), dtype=torch.float32, device=dev)
    L.check(lib.edt_slerp_refdot(L.ptr(v0), L.ptr(v1), L.dtype_code(v0), L.ptr(chunks), nchunks, L.ptr(seg_first),
                                 nseg, int(chunk_elems), L.ptr(flag), int(ref.threads), float(eps), L.ptr(val),
                                 L.ptr(ws), ws.numel() * 8, L.stream_ptr(dev)), "edt_slerp_refdot")
    return val


def slerp_population(plan: SlerpPlan, members: list[torch.Tensor], pairs, outs: list[torch.Tensor],
                     t: torch.Tensor, dot_threshold: float = 0.9995, eps: float = 1e-8,
                     speculate: bool | None = None, ref_dot: RefDot | None = None) -> torch.Tensor:
    """SLERP child q of members[pairs[q][0]], members[pairs[q][1]] into outs[q], for every q
    (EDT_RL/edt.py:286-299 -> EDT_RL/crossover.py:84-135 per child). Two forms, bit-identical to
    slerp_arena per child:
      speculate=False  edt_slerp_population: one stats pass per component of the children's
                       pair graph over the (<= 8) distinct parents (r5: the needed sums — each
                       parent's norm and only the dots its children use, for any graph the
                       reference's selection draws; r6: the same pass in the triangle layout
                       — the component's Gram triangle, unused dots skipped — when it needs more
                       dots than its slots), then one member-major blend launch for all children;
      speculate=True   edt_slerp_population_speculative: one pass forms every child's sums and
                       writes its lerp-branch output (r5: a member-major needed-sums pass per
                       component when every component takes the needed layout and there are <= 16
                       children; else the co-located pass), then only SLERP-branch segments are
                       blended again (parents of one lineage: a single pass);
      None             speculate when the previous call on this plan had few enough child elements
                       in SLERP-branch segments for the single pass to move fewer bytes
                       (f < D b_in / (D b_in + Q b_out), D distinct parents, Q children).
    ref_dot: the reference-dot mode per child (as slerp_arena's; the two-pass form runs its passes
    separately: needed sums -> coefficients' dots -> the reference's dots and coefficients ->
    blends).
    Returns the per-child, per-segment fp32 dots ([npairs, nseg])."""
    lib = L.lib()
    M, Q = len(members), len(pairs)
    if plan.relative:
        raise L.EdtError("slerp_population runs over flat member arenas (a non-relative plan)")
    if len(outs) != Q:
        raise L.EdtError("one output per pair")
    L.require_device(*members, *outs, t)
    n = plan.seg_offsets[-1]
    in_dt, out_dt = members[0].dtype, outs[0].dtype if outs else members[0].dtype
    if any(m.dtype != in_dt or m.numel() != n for m in members) or any(o.dtype != out_dt or o.numel() != n for o in outs):
        raise L.EdtError("members / outputs must match the plan's layout and share one dtype each")
    if t.dtype != torch.float64 or t.numel() < plan.nseg:
        raise L.EdtError("t must be a float64 device tensor with one value per segment")
    if speculate is None:
        d = _host_dots(plan, "_pop_dots", wait=False) if getattr(plan, "_last_thr", None) is not None else None
        if getattr(plan, "_pop_dots", None) is None or getattr(plan, "_last_thr", None) is None:
            speculate = True
        elif d is None or d.shape[0] == 0:        # previous dots still in flight: keep its decision
            speculate = getattr(plan, "_last_pop_speculate", True)
        else:
            import numpy as np
            sizes = np.diff(np.asarray(plan.seg_offsets, dtype=np.int64))
            f = float((sizes[None, :] * (np.abs(d) <= plan._last_thr)).sum()) / max(1, int(sizes.sum()) * d.shape[0])
            # member-major passes over D distinct parents: speculating costs (1 + f)(D b_in + Q b_out)
            # against 2 D b_in + Q b_out for the Gram form
            D = len({int(x) for p in pairs for x in p})
            bi, bo = members[0].element_size(), (outs[0].element_size() if outs else members[0].element_size())
            speculate = f < D * bi / max(1, D * bi + Q * bo)
        plan._last_pop_speculate = speculate
    if any(_overlap(o, m) for o in outs for m in members):
        speculate = False
    if not speculate and not 1 <= M <= 8:
        raise L.EdtError(f"the Gram form takes 1..8 members, got {M}")
    dev = t.device
    coef = torch.empty((max(1, Q), max(1, plan.nseg), 2), dtype=torch.float32, device=dev)
    dots = torch.empty((max(1, Q), max(1, plan.nseg)), dtype=torch.float32, device=dev)
    flat_pairs = (ctypes.c_int32 * max(1, 2 * Q))(*[int(x) for p in pairs for x in p])
    icode, ocode = L.dtype_code(in_dt), L.dtype_code(out_dt)
    if ref_dot is not None and not speculate and Q:
        # the two-pass form's passes separately: sums -> dots -> the reference's coefficients -> blends
        layout = needed_table(pairs, M, plan.nchunks)
        table = plan.ws("needed", max(1, layout.doubles), torch.float64)
        slerp_needed_sums(members, layout, plan.chunks, plan.nchunks, table, 0)
        _, dots = slerp_needed_coef(plan, table, layout, t, dot_threshold, eps)
        dots, coef = _population_ref(plan, members, pairs, outs, t, dots, None, icode, ocode, dot_threshold, eps,
                                     ref_dot, blend_all=True)
    elif speculate:
        part = _scratch(dev, int(lib.edt_slerp_population_speculative_doubles(Q, plan.nchunks)))
        redo = torch.empty(max(1, Q * plan.nseg), dtype=torch.int32, device=dev)
        L.check(lib.edt_slerp_population_speculative(
            L.ptr_array(members), M, icode, flat_pairs, Q, L.ptr_array(outs), ocode,
            L.ptr(plan.chunks), plan.nchunks, L.ptr(plan.seg_first), plan.nseg, L.ptr(t), float(dot_threshold),
            float(eps), L.ptr(part), L.ptr(coef), L.ptr(dots), L.ptr(redo), n, L.stream_ptr(dev)),
            "edt_slerp_population_speculative")
        if ref_dot is not None and Q:
            dots, coef = _population_ref(plan, members, pairs, outs, t, dots, coef, icode, ocode, dot_threshold, eps,
                                         ref_dot, blend_all=False)
    else:
        gram = plan.ws("gram", int(lib.edt_slerp_population_gram_doubles(M, plan.nchunks)), torch.float64)
        L.check(lib.edt_slerp_population(L.ptr_array(members), M, icode, flat_pairs, Q,
                                         L.ptr_array(outs), ocode, L.ptr(plan.chunks), plan.nchunks,
                                         L.ptr(plan.seg_first), plan.nseg, L.ptr(t), float(dot_threshold), float(eps),
                                         L.ptr(gram), L.ptr(coef), L.ptr(dots), L.stream_ptr(dev)),
                "edt_slerp_population")
    dots = dots[:Q, :plan.nseg]
    plan._pop_dots = dots                        # the latest generation's (bench.py reads it)
    plan._last_thr = float(dot_threshold)
    _record_dots(plan, dots, "_pop_dots")
    return dots


def pair_merge_population(children, lr: float, momentum_coef: float, nesterov: bool) -> None:
    """Every EDT-LM child of a resident population in one launch (edt_pair_merge_population).
    children: dicts with b1, b2, m1, m2 (parent arenas, repeated across children), out, and
    momentum_in / momentum (the donor's buffer, read; the child's, written) / has_momentum.
    Bit-identical to pair_merge(..., momentum_in=...) per child; parents shared by several
    children cross HBM once (same-XCD workgroups, cache reuse)."""
    lib = L.lib()
    C = len(children)
    if not 1 <= C <= 16:
        raise L.EdtError(f"pair_merge_population takes 1..16 children, got {C} (use pair_merge per child)")
    first = children[0]
    n = first["out"].numel()
    wdt, gdt = first["m1"].dtype, first["out"].dtype
    for ch in children:
        ts = [ch[k] for k in ("b1", "b2", "m1", "m2", "out")] + [ch.get("momentum"), ch.get("momentum_in")]
        L.require_device(*ts)
        if any(t is not None and t.numel() != n for t in ts):
            raise L.EdtError("pair-merge buffers must all have the same size")
        if any(ch[k].dtype != wdt for k in ("b1", "b2", "m1", "m2")) or ch["out"].dtype != gdt:
            raise L.EdtError("one parent dtype and one child dtype for the whole population")
        if any(ch.get(k) is not None and ch[k].dtype != gdt for k in ("momentum", "momentum_in")):
            raise L.EdtError("momentum buffers must have the child's dtype")
    has = (ctypes.c_int32 * C)(*[int(bool(ch.get("has_momentum"))) for ch in children])
    mom_out = [ch.get("momentum") for ch in children]
    mom_in = [ch.get("momentum_in") if ch.get("has_momentum") else None for ch in children]
    arr = lambda ts: (ctypes.c_void_p * C)(*[0 if t is None else t.data_ptr() for t in ts])
    L.check(lib.edt_pair_merge_population(
        L.ptr_array([ch["b1"] for ch in children]), L.ptr_array([ch["b2"] for ch in children]),
        L.ptr_array([ch["m1"] for ch in children]), L.ptr_array([ch["m2"] for ch in children]),
        L.dtype_code(wdt), L.ptr_array([ch["out"] for ch in children]), L.dtype_code(gdt),
        arr(mom_in), arr(mom_out), has, C, n, float(lr), float(momentum_coef), int(nesterov),
        L.stream_ptr(first["out"].device)), "edt_pair_merge_population")


# ------------------------------------------------------------------------------------------
# the population SLERP's passes, separately (distributed.ShardedPopulationCrossover)

@dataclass(frozen=True)
class NeededTable:
    """The needed-sums table of one generation (edt_slerp_needed_table, host only): the pair graph's
    components as blocks of `nchunks` rows, block k at blocks[k][0] doubles with blocks[k][1] sums
    per row; columns[k][c] = the two members column c of block k sums over ((-1, -1): unused)."""
    pairs: tuple
    nmembers: int
    nchunks: int
    blocks: tuple
    columns: tuple
    doubles: int
    scratch_doubles: int

    def rows(self, table: torch.Tensor, k: int, a: int, b: int) -> torch.Tensor:
        """Rows [a, b) of block k (a contiguous view of the table)."""
        off, nt = self.blocks[k]
        return table[off + a * nt:off + b * nt]


_needed_memo: dict = {}


def needed_table(pairs, nmembers: int, nchunks: int) -> NeededTable:
    """The table layout the needed-sums passes use for these pairs (cached)."""
    key = (tuple((int(a), int(b)) for a, b in pairs), int(nmembers), int(nchunks))
    got = _needed_memo.get(key)
    if got is not None:
        return got
    lib = L.load_library()
    Q = len(key[0])
    fp = (ctypes.c_int32 * max(1, 2 * Q))(*[x for p in key[0] for x in p])
    off = (ctypes.c_uint64 * 8)()
    nt = (ctypes.c_int32 * 8)()
    nc = ctypes.c_int32()
    cols = (ctypes.c_int32 * (2 * 36 * 8))()
    tot, scr = ctypes.c_uint64(), ctypes.c_uint64()
    L.check(lib.edt_slerp_needed_table(fp, Q, key[1], key[2], off, nt, ctypes.byref(nc), cols, ctypes.byref(tot),
                                       ctypes.byref(scr)), "edt_slerp_needed_table")
    blocks, columns, c = [], [], 0
    for k in range(nc.value):
        blocks.append((int(off[k]), int(nt[k])))
        columns.append(tuple((int(cols[2 * (c + x)]), int(cols[2 * (c + x) + 1])) for x in range(nt[k])))
        c += nt[k]
    got = NeededTable(key[0], key[1], key[2], tuple(blocks), tuple(columns), int(tot.value), int(scr.value))
    if len(_needed_memo) > 64:
        _needed_memo.clear()
    _needed_memo[key] = got
    return got


def slerp_needed_sums(members: list[torch.Tensor], layout: NeededTable, chunks: torch.Tensor, nchunks: int,
                      table: torch.Tensor, row0: int, scratch: torch.Tensor | None = None) -> torch.Tensor:
    """Rows [row0, row0 + nchunks) of every block of `layout`'s table (float64, >= layout.doubles)
    over a chunk table of those chunks (starts relative to the member buffers):
    edt_slerp_needed_sums. `scratch`: >= layout.scratch_doubles float64 (default: the stream's
    pooled workspace)."""
    lib = L.lib()
    M = len(members)
    if M != layout.nmembers:
        raise L.EdtError("slerp_needed_sums: one buffer per member of the layout")
    L.require_device(*members, chunks, table)
    if table.dtype != torch.float64 or table.numel() < layout.doubles or not table.is_contiguous():
        raise L.EdtError("table: contiguous float64 with the layout's doubles")
    need = max(1, layout.scratch_doubles)
    if scratch is None or scratch.dtype != torch.float64 or scratch.numel() < need:
        scratch = _scratch(members[0].device, need)
    Q = len(layout.pairs)
    fp = (ctypes.c_int32 * max(1, 2 * Q))(*[x for p in layout.pairs for x in p])
    L.check(lib.edt_slerp_needed_sums(L.ptr_array(members), M, L.dtype_code(members[0]), fp, Q, L.ptr(chunks),
                                      int(nchunks), layout.nchunks, int(row0), L.ptr(table), L.ptr(scratch),
                                      scratch.numel(), L.stream_ptr(members[0].device)), "edt_slerp_needed_sums")
    return table


def slerp_needed_coef(plan: SlerpPlan, table: torch.Tensor, layout: NeededTable, t: torch.Tensor,
                      dot_threshold: float = 0.9995, eps: float = 1e-8):
    """Coefficients [Q, nseg, 2] and dots [Q, nseg] of every child of `layout` from its complete
    table (rows = plan's chunks): edt_slerp_needed_coef."""
    lib = L.lib()
    Q = len(layout.pairs)
    if layout.nchunks != plan.nchunks or table.numel() < layout.doubles:
        raise L.EdtError("the table does not cover the plan's chunks")
    L.require_device(table, t)
    if t.dtype != torch.float64 or t.numel() < plan.nseg:
        raise L.EdtError("t must be a float64 device tensor with one value per segment")
    dev = table.device
    coef = torch.empty((max(1, Q), max(1, plan.nseg), 2), dtype=torch.float32, device=dev)
    dots = torch.empty((max(1, Q), max(1, plan.nseg)), dtype=torch.float32, device=dev)
    fp = (ctypes.c_int32 * max(1, 2 * Q))(*[x for p in layout.pairs for x in p])
    L.check(lib.edt_slerp_needed_coef(L.ptr(table), layout.nchunks, fp, Q, layout.nmembers, L.ptr(plan.seg_first),
                                      plan.nseg, L.ptr(t), float(dot_threshold), float(eps), L.ptr(coef), L.ptr(dots),
                                      L.stream_ptr(dev)), "edt_slerp_needed_coef")
    return coef, dots


def slerp_blend_children(members: list[torch.Tensor], pairs, outs: list[torch.Tensor], chunks: torch.Tensor,
                         nchunks: int, coef: torch.Tensor, nseg: int) -> None:
    """outs[q] = c0 members[a] + c1 members[b] over a chunk table, coef [Q, nseg, 2] per child
    (edt_slerp_blend_children; <= 8 members, <= 16 children)."""
    lib = L.lib()
    Q = len(pairs)
    L.require_device(*members, *outs, chunks, coef)
    if Q != len(outs) or coef.dtype != torch.float32 or coef.numel() < Q * nseg * 2:
        raise L.EdtError("slerp_blend_children: one output per pair, coef [Q, nseg, 2] float32")
    fp = (ctypes.c_int32 * max(1, 2 * Q))(*[int(x) for p in pairs for x in p])
    L.check(lib.edt_slerp_blend_children(L.ptr_array(members), len(members), L.dtype_code(members[0]), fp, Q,
                                         L.ptr_array(outs), L.dtype_code(outs[0]), L.ptr(chunks), nchunks,
                                         L.ptr(coef), nseg, L.stream_ptr(members[0].device)),
            "edt_slerp_blend_children")


def population_layout(pairs, nmembers: int, speculate: bool = True) -> dict:
    """How edt_slerp_population(_speculative) lays out a generation for these pairs — the
    library's own planner (edt_slerp_population_layout, host only): the form ("member-major" /
    "co-located" speculative, "two-pass"), and per component of the children's pair graph its
    members, distinct dots, sums per element and stats layout ("needed" / "triangle")."""
    import json as _json
    lib = L.load_library()
    Q = len(pairs)
    fp = (ctypes.c_int32 * max(1, 2 * Q))(*[int(x) for p in pairs for x in p])
    buf = ctypes.create_string_buffer(8192)
    L.check(lib.edt_slerp_population_layout(fp, Q, int(nmembers), int(bool(speculate)), buf, len(buf)),
            "edt_slerp_population_layout")
    return _json.loads(buf.value.decode())
