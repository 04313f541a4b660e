"""Flat-buffer operators: one call = one fused HIP launch over a whole parameter arena.

Every function takes device-resident, contiguous tensors (flat views of the population's
parameter arenas, see `params.ParamArena`) and launches on the current HIP stream. Nothing here
synchronises, allocates persistent memory or falls back to the CPU: a missing library or device
raises `EdtError`.
"""
from __future__ import annotations

import ctypes
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
                    momentum_coef: float, nesterov: bool) -> None:
    """`outer_step` over T separate tensors per model (e.g. `list(model.parameters())` of
    models loaded on the GPU) in ONE launch, without packing: thetas[t], workers[k][t],
    momenta[t] (theta's dtype, required when momentum_coef != 0), all updated in place."""
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
    L.check(lib.edt_outer_step_list(th_arr, L.dtype_code(gdt), w_arr, L.dtype_code(wdt), K, m_arr,
                                    int(has_momentum), numel, T, float(lr), float(momentum_coef), int(nesterov),
                                    L.ptr(ws), nbytes, L.stream_ptr(thetas[0].device)), "edt_outer_step_list")


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

@dataclass
class SlerpPlan:
    """Chunk table for a segment layout, resident on the device (built once per layout)."""
    seg_offsets: list[int]
    chunks: torch.Tensor          # int64 [nchunks, 3] = start, length, segment
    seg_first: torch.Tensor       # int32 [nseg + 1]
    partial: torch.Tensor         # float64 workspace: chunk rows [nchunks, 3], then the slot scratch
    coef: torch.Tensor            # float32 [nseg, 2]
    dots: torch.Tensor            # float32 [nseg]
    nchunks: int
    relative: bool = False        # chunk starts relative to their segment (tensor-list form)
    chunks_host: object = None    # numpy int64 [nchunks, 3]: the same table on the host
    chunk_elems: int = 1 << 16

    @property
    def nseg(self) -> int:
        return len(self.seg_offsets) - 1


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
    return SlerpPlan(list(seg_offsets), chunks, seg_first,
                     torch.empty(max(1, int(lib.edt_slerp_sums_doubles(3, nchunks))), dtype=torch.float64,
                                 device=device),
                     torch.empty((max(1, nseg), 2), dtype=torch.float32, device=device),
                     torch.empty(max(1, nseg), dtype=torch.float32, device=device), nchunks, relative, host,
                     int(chunk_elems))


@dataclass(frozen=True)
class RefDot:
    """Reference-dot mode for the SLERP branch decision (include/edt_sync.h, edt_slerp_refdot):
    segments whose fp64 dot lies within `band` of DOT_THRESHOLD (band < 0: every segment) take the
    reference's own fp32 dot — BLAS sdot norms + numpy's pairwise sum, restated bit for bit for
    the reference host's numpy / OpenBLAS (`threads` = OpenBLAS's thread count for sdot there; 1 on
    the pinned host) — and the branch and coefficients that follow from it. Without it (the
    default) the kernels decide from their fp64 dot, the accurate one."""
    threads: int = 1
    band: float = -1.0


def _refdot_pass(plan: SlerpPlan, v0: torch.Tensor, v1: torch.Tensor, t: torch.Tensor, dot_threshold: float,
                 eps: float, ref: RefDot) -> None:
    """After edt_slerp_coef: flag segments, recompute their dot the reference's way, overwrite
    their coefficients and dots (plan.coef / plan.dots)."""
    lib = L.lib()
    dev, st = v0.device, L.stream_ptr(v0.device)
    need = int(lib.edt_slerp_refdot_workspace_bytes(plan.nseg, plan.nchunks, plan.chunk_elems, int(ref.threads)))
    if need == 0:
        raise L.EdtError(f"reference-dot mode needs chunks of a multiple of 8192 elements (plan: {plan.chunk_elems})")
    ws = getattr(plan, "_refdot_ws", None)
    if ws is None or ws.numel() * 8 < need:
        ws = plan._refdot_ws = torch.empty((need + 7) // 8, dtype=torch.float64, device=dev)
        plan._refdot_flag = torch.empty(max(1, plan.nseg), dtype=torch.int32, device=dev)
        plan._refdot_val = torch.empty(max(1, plan.nseg), dtype=torch.float32, device=dev)
    L.check(lib.edt_slerp_refdot_flags(L.ptr(plan.dots), plan.nseg, float(dot_threshold), float(ref.band),
                                       L.ptr(plan._refdot_flag), st), "edt_slerp_refdot_flags")
    L.check(lib.edt_slerp_refdot(L.ptr(v0), L.ptr(v1), L.dtype_code(v0), L.ptr(plan.chunks), plan.nchunks,
                                 L.ptr(plan.seg_first), plan.nseg, plan.chunk_elems, L.ptr(plan._refdot_flag),
                                 int(ref.threads), float(eps), L.ptr(plan._refdot_val), L.ptr(ws), ws.numel() * 8, st),
            "edt_slerp_refdot")
    L.check(lib.edt_slerp_refdot_coef(L.ptr(plan._refdot_val), L.ptr(plan._refdot_flag), plan.nseg, L.ptr(t),
                                      float(dot_threshold), L.ptr(plan.coef), L.ptr(plan.dots), st),
            "edt_slerp_refdot_coef")


def _record_dots(plan: SlerpPlan, dots: torch.Tensor, attr: str) -> None:
    """After a merge: the dots go to pinned host memory by an async copy on the merge's stream, with
    an event, so the next call can judge its form without synchronising the device."""
    host = getattr(plan, attr + "_host", None)
    if host is None or host.shape != dots.shape:
        host = torch.empty(dots.shape, dtype=dots.dtype, pin_memory=True)
        setattr(plan, attr + "_host", host)
    host.copy_(dots, non_blocking=True)
    ev = torch.cuda.Event()
    ev.record(torch.cuda.current_stream(dots.device))
    setattr(plan, attr + "_event", ev)


def _host_dots(plan: SlerpPlan, attr: str, wait: bool):
    """The previous merge's dots on the host (numpy), or None while its copy is still in flight
    (wait=False: never blocks; wait=True: waits for that copy only)."""
    ev = getattr(plan, attr + "_event", None)
    if ev is None:
        return None
    if wait:
        ev.synchronize()
    elif not ev.query():
        return None
    return getattr(plan, attr + "_host").numpy()


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
    sizes = np.diff(np.asarray(plan.seg_offsets, dtype=np.int64))
    total = max(1, int(sizes.sum()))
    f = float(sizes[np.abs(dots) <= plan._last_thr].sum()) / total
    return (1 + f) * (2 * in_bytes + out_bytes) < 4 * in_bytes + out_bytes


def _overlap(a: torch.Tensor, b: torch.Tensor) -> bool:
    a0, b0 = a.data_ptr(), b.data_ptr()
    return a0 < b0 + b.numel() * b.element_size() and b0 < a0 + a.numel() * a.element_size()


def slerp_arena(plan: SlerpPlan, v0: torch.Tensor, v1: torch.Tensor, out: torch.Tensor,
                t: torch.Tensor, dot_threshold: float = 0.9995, eps: float = 1e-8,
                speculate: bool | None = None, ref_dot: RefDot | None = None) -> None:
    """SLERP every segment of v0/v1 with its own t (float64 device tensor [nseg]) into out
    (EDT_RL/crossover.py:11-43): chunk sums, per-segment coefficients, blend (edt_slerp_merge).
    speculate: True = edt_slerp_merge_speculative (lerp-branch output written in the stats pass,
    only SLERP-branch segments blended again); False = the two-pass form; None = whichever the
    previous merge on this plan says is cheaper. Bit-identical results either way; an output
    that overlaps a parent always takes the two-pass form. ref_dot (RefDot): the reference-dot
    mode, always the split two-pass form: stats -> coef -> refdot -> blend."""
    lib = L.lib()
    L.require_device(v0, v1, out, t)
    if v1.dtype != v0.dtype or v0.numel() != plan.seg_offsets[-1] or v1.numel() != v0.numel() \
            or out.numel() != v0.numel():
        raise L.EdtError("slerp arenas must match the plan's layout")
    if t.dtype != torch.float64 or t.numel() < plan.nseg:
        raise L.EdtError("t must be a float64 device tensor with one value per segment")
    if plan.relative:
        raise L.EdtError("a relative (tensor-list) plan drives slerp_list, not slerp_arena")
    if ref_dot is not None:
        st = L.stream_ptr(v0.device)
        L.check(lib.edt_slerp_stats(L.ptr(v0), L.ptr(v1), L.dtype_code(v0), L.ptr(plan.chunks), plan.nchunks,
                                    L.ptr(plan.partial), st), "edt_slerp_stats")
        L.check(lib.edt_slerp_coef(L.ptr(plan.partial), L.ptr(plan.seg_first), plan.nseg, L.ptr(t),
                                   float(dot_threshold), float(eps), L.ptr(plan.coef), L.ptr(plan.dots), st),
                "edt_slerp_coef")
        _refdot_pass(plan, v0, v1, t, dot_threshold, eps, ref_dot)
        L.check(lib.edt_slerp_blend(L.ptr(v0), L.ptr(v1), L.dtype_code(v0), L.ptr(out), L.dtype_code(out),
                                    L.ptr(plan.chunks), plan.nchunks, L.ptr(plan.coef), st), "edt_slerp_blend")
        plan._last_thr = float(dot_threshold)
        _record_dots(plan, plan.dots[:max(1, plan.nseg)], "_dots")
        return
    if speculate is None:
        speculate = _speculation_pays(plan, v0.element_size(), out.element_size(), wait=False)
        plan._last_speculate = speculate
    if speculate and (_overlap(out, v0) or _overlap(out, v1)):
        speculate = False
    if speculate:
        redo = getattr(plan, "_redo", None)
        if redo is None:
            redo = plan._redo = torch.empty(max(1, plan.nseg), dtype=torch.int32, device=v0.device)
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


def _spans_apart(out_ptrs, out_bytes, in_ptrs, in_bytes) -> bool:
    """No output span [ptr, ptr + bytes) overlaps an input span: spans sorted by start, each checked
    against the furthest end of the other kind before it (numpy; empty spans ignored)."""
    import numpy as np
    a = np.concatenate((np.asarray(in_ptrs, dtype=np.int64), np.asarray(out_ptrs, dtype=np.int64)))
    n = np.concatenate((np.asarray(in_bytes, dtype=np.int64), np.asarray(out_bytes, dtype=np.int64)))
    k = np.concatenate((np.zeros(len(in_ptrs), dtype=bool), np.ones(len(out_ptrs), dtype=bool)))
    keep = n > 0
    a, n, k = a[keep], n[keep], k[keep]
    if a.size == 0:
        return True
    o = np.argsort(a, kind="stable")
    a, e, k = a[o], a[o] + n[o], k[o]
    far_out = np.maximum.accumulate(np.where(k, e, -1))       # furthest end of an output so far
    far_in = np.maximum.accumulate(np.where(k, -1, e))
    prev_out = np.concatenate(([-1], far_out[:-1]))
    prev_in = np.concatenate(([-1], far_in[:-1]))
    return not bool(np.any(np.where(k, a < prev_in, a < prev_out)))


def slerp_list(plan: SlerpPlan, v0s: list[torch.Tensor], v1s: list[torch.Tensor], outs: list[torch.Tensor],
               t: torch.Tensor, dot_threshold: float = 0.9995, eps: float = 1e-8,
               speculate: bool | None = None) -> None:
    """`slerp_arena` over separate tensors (one segment each, e.g. two models' state-dict
    tensors), writing straight into `outs` (e.g. the target model's parameters): no packing.
    Every tensor must be contiguous and 16-byte aligned; plan = make_slerp_plan(...,
    relative=True) over the tensors' sizes. speculate as slerp_arena's: True =
    edt_slerp_merge_list_speculative (lerp-branch outputs written in the sums pass, only
    SLERP-branch tensors blended again), False = the two-pass edt_slerp_merge_list, None = the
    cheaper by the previous merge's dots on this plan; outputs that overlap a parent (e.g. merged
    into the first parent's own tensors) always take the two-pass form. Bit-identical either way."""
    lib = L.lib()
    T = len(v0s)
    if not plan.relative or T != plan.nseg or len(v1s) != T or len(outs) != T:
        raise L.EdtError("slerp_list needs a relative plan with one segment per tensor")
    L.require_device(*v0s, *v1s, *outs, t)
    in_dt, out_dt = v0s[0].dtype, outs[0].dtype
    for i in range(T):
        n = plan.seg_offsets[i + 1] - plan.seg_offsets[i]
        if v0s[i].numel() != n or v1s[i].numel() != n or outs[i].numel() != n:
            raise L.EdtError(f"tensor {i} does not match the plan's layout")
        if v0s[i].dtype != in_dt or v1s[i].dtype != in_dt or outs[i].dtype != out_dt:
            raise L.EdtError("slerp_list: one input dtype and one output dtype")
    if t.dtype != torch.float64 or t.numel() < T:
        raise L.EdtError("t must be a float64 device tensor with one value per segment")
    ws = torch.empty(max(1, 3 * T), dtype=torch.int64, device=t.device)
    p0, p1, po = ([x.data_ptr() for x in ts] for ts in (v0s, v1s, outs))
    if speculate is None:
        speculate = _speculation_pays(plan, v0s[0].element_size(), outs[0].element_size(), wait=False)
        plan._last_speculate = speculate
    if speculate:
        import numpy as np
        n = np.diff(np.asarray(plan.seg_offsets, dtype=np.int64))
        nin, nout = n * v0s[0].element_size(), n * outs[0].element_size()
        speculate = _spans_apart(po, nout, p0 + p1, np.concatenate((nin, nin)))
    tab = [(ctypes.c_void_p * max(1, T))(*p) for p in (p0, p1, po)]
    st = L.stream_ptr(t.device)
    if speculate:
        redo = getattr(plan, "_redo", None)
        if redo is None:
            redo = plan._redo = torch.empty(max(1, plan.nseg), dtype=torch.int32, device=t.device)
        L.check(lib.edt_slerp_merge_list_speculative(
            tab[0], tab[1], L.dtype_code(in_dt), tab[2], L.dtype_code(out_dt),
            L.ptr(plan.chunks), plan.nchunks, L.ptr(plan.seg_first), T, L.ptr(t), float(dot_threshold), float(eps),
            L.ptr(plan.partial), L.ptr(plan.coef), L.ptr(plan.dots), L.ptr(redo), L.ptr(ws), ws.numel() * 8, st),
            "edt_slerp_merge_list_speculative")
    else:
        L.check(lib.edt_slerp_merge_list(tab[0], tab[1], L.dtype_code(in_dt),
                                         tab[2], L.dtype_code(out_dt), L.ptr(plan.chunks), plan.nchunks,
                                         L.ptr(plan.seg_first), T, L.ptr(t), float(dot_threshold), float(eps),
                                         L.ptr(plan.partial), L.ptr(plan.coef), L.ptr(plan.dots), L.ptr(ws),
                                         ws.numel() * 8, st), "edt_slerp_merge_list")
    plan._last_thr = float(dot_threshold)
    _record_dots(plan, plan.dots[:max(1, plan.nseg)], "_dots")


def slerp_population(plan: SlerpPlan, members: list[torch.Tensor], pairs, outs: list[torch.Tensor],
                     t: torch.Tensor, dot_threshold: float = 0.9995, eps: float = 1e-8,
                     speculate: bool | None = None) -> torch.Tensor:
    """SLERP child q of members[pairs[q][0]], members[pairs[q][1]] into outs[q], for every q
    (EDT_RL/edt.py:286-299 -> EDT_RL/crossover.py:84-135 per child). Two forms, bit-identical to
    slerp_arena per child:
      speculate=False  edt_slerp_population: ONE Gram stats pass over the (<= 8) members, then
                       one co-located blend launch for all children;
      speculate=True   edt_slerp_population_speculative: one co-located pass forms every child's
                       sums and writes its lerp-branch output, then only SLERP-branch segments
                       are blended again (parents of one lineage: a single pass);
      None             speculate when the previous call on this plan had few enough child elements
                       in SLERP-branch segments for the single pass to move fewer bytes
                       (f < D b_in / (D b_in + Q b_out), D distinct parents, Q children).
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
    if speculate:
        part = torch.empty(max(1, int(lib.edt_slerp_population_speculative_doubles(Q, plan.nchunks))),
                           dtype=torch.float64, device=dev)
        redo = torch.empty(max(1, Q * plan.nseg), dtype=torch.int32, device=dev)
        L.check(lib.edt_slerp_population_speculative(
            L.ptr_array(members), M, L.dtype_code(in_dt), flat_pairs, Q, L.ptr_array(outs), L.dtype_code(out_dt),
            L.ptr(plan.chunks), plan.nchunks, L.ptr(plan.seg_first), plan.nseg, L.ptr(t), float(dot_threshold),
            float(eps), L.ptr(part), L.ptr(coef), L.ptr(dots), L.ptr(redo), n, L.stream_ptr(dev)),
            "edt_slerp_population_speculative")
    else:
        need = int(lib.edt_slerp_population_gram_doubles(M, plan.nchunks))
        gram = getattr(plan, "_gram", None)
        if gram is None or gram.numel() < max(1, need):
            gram = plan._gram = torch.empty(max(1, need), dtype=torch.float64, device=dev)
        L.check(lib.edt_slerp_population(L.ptr_array(members), M, L.dtype_code(in_dt), flat_pairs, Q,
                                         L.ptr_array(outs), L.dtype_code(out_dt), L.ptr(plan.chunks), plan.nchunks,
                                         L.ptr(plan.seg_first), plan.nseg, L.ptr(t), float(dot_threshold), float(eps),
                                         L.ptr(gram), L.ptr(coef), L.ptr(dots), L.stream_ptr(dev)),
                "edt_slerp_population")
    plan._pop_dots = dots[:Q, :plan.nseg]
    plan._last_thr = float(dot_threshold)
    _record_dots(plan, plan._pop_dots, "_pop_dots")
    return plan._pop_dots


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
# the population SLERP's three passes, separately (distributed.ShardedSlerpPopulation)

def slerp_gram(members: list[torch.Tensor], chunks: torch.Tensor, nchunks: int,
               gram: torch.Tensor | None = None) -> torch.Tensor:
    """Per-chunk Gram sums of M <= 8 member buffers over a chunk table (int64 [nchunks, 3] on the
    device, starts relative to the buffers): float64 [nchunks, M(M+1)/2] (edt_slerp_gram). `gram`
    (optional) receives the rows; its first nchunks x M(M+1)/2 elements are written."""
    lib = L.lib()
    M = len(members)
    L.require_device(*members, chunks)
    if not 1 <= M <= 8 or any(m.dtype != members[0].dtype for m in members):
        raise L.EdtError("slerp_gram: 1..8 members of one dtype")
    NT = M * (M + 1) // 2
    need = max(1, int(lib.edt_slerp_population_gram_doubles(M, nchunks)))
    if gram is not None and (gram.dtype != torch.float64 or gram.numel() < nchunks * NT):
        raise L.EdtError("gram: float64 with nchunks x M(M+1)/2 elements")
    # the kernel needs the rows plus its slot scratch behind them; a smaller (or non-contiguous)
    # `gram` — e.g. a rank's rows of the whole table — gets its rows copied from a full-size buffer
    direct = gram is not None and gram.is_contiguous() and gram.numel() >= need
    work = gram if direct else torch.empty(need, dtype=torch.float64, device=members[0].device)
    L.check(lib.edt_slerp_gram(L.ptr_array(members), M, L.dtype_code(members[0]), L.ptr(chunks), nchunks,
                               L.ptr(work), L.stream_ptr(members[0].device)), "edt_slerp_gram")
    rows = work.view(-1)[:nchunks * NT].view(nchunks, NT) if not direct else gram
    if gram is None:
        return rows
    if not direct:
        gram.view(-1)[:nchunks * NT].copy_(rows.view(-1))
    return gram


def slerp_gram_coef(plan: SlerpPlan, gram: torch.Tensor, nmembers: int, pairs, t: torch.Tensor,
                    dot_threshold: float = 0.9995, eps: float = 1e-8):
    """Coefficients [Q, nseg, 2] and dots [Q, nseg] of every child from a whole-layout Gram
    table (rows = plan's chunks) (edt_slerp_gram_coef)."""
    lib = L.lib()
    Q = len(pairs)
    if gram.numel() < plan.nchunks * nmembers * (nmembers + 1) // 2:
        raise L.EdtError("gram does not cover the plan's chunks")
    L.require_device(gram, t)
    if t.dtype != torch.float64 or t.numel() < plan.nseg:
        raise L.EdtError("t must be a float64 device tensor with one value per segment")
    dev = gram.device
    coef = torch.empty((max(1, Q), max(1, plan.nseg), 2), dtype=torch.float32, device=dev)
    dots = torch.empty((max(1, Q), max(1, plan.nseg)), dtype=torch.float32, device=dev)
    fp = (ctypes.c_int32 * max(1, 2 * Q))(*[int(x) for p in pairs for x in p])
    L.check(lib.edt_slerp_gram_coef(L.ptr(gram), nmembers, fp, Q, L.ptr(plan.seg_first), plan.nseg, L.ptr(t),
                                    float(dot_threshold), float(eps), L.ptr(coef), L.ptr(dots),
                                    L.stream_ptr(dev)), "edt_slerp_gram_coef")
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
