"""CPU oracle for the outer-loop sync hot path — TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's `cpu_baseline` leg import this module, and
only as the checker / the timed CPU baseline. The product package never imports it.

Two parts:
  * ctypes wrappers over oracle/_build/liboracle.so (edt_oracle.c): the DiLoCo outer step, the
    EDT pair merge and lerp, restated element by element in the reference's torch op order.
  * a numpy restatement of the SLERP crossover (EDT_RL/crossover.py:11-81,
    EDT_EVOMERGE/train/crossover.py:14-83): same numpy primitives in the same order, so it is
    bit-exact with the reference on the same inputs (pinned by tests/test_oracle_golden.py).

All tensors are CPU torch tensors (float32 or bfloat16), contiguous; updates happen in place.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "_build", "liboracle.so")

F32, BF16 = 0, 1
_DT = {torch.float32: F32, torch.bfloat16: BF16}
_P, _U64, _I, _D = ctypes.c_void_p, ctypes.c_uint64, ctypes.c_int, ctypes.c_double
_lib = None


def build() -> str:
    """Compile liboracle.so (gcc) if it is missing or older than its source."""
    src = os.path.join(HERE, "edt_oracle.c")
    if not os.path.exists(LIB) or os.path.getmtime(LIB) < os.path.getmtime(src):
        subprocess.run(["make", "-C", HERE, "-s"], check=True)
    return LIB


def lib() -> ctypes.CDLL:
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            build()
        l = ctypes.CDLL(LIB)
        l.oracle_outer_step.argtypes = [_P, _I, ctypes.POINTER(_P), _I, _I, _P, _I, _U64, _D, _D, _I, _P]
        l.oracle_pair_merge.argtypes = [_P, _P, _P, _P, _I, _P, _I, _P, _I, _U64, _D, _D, _I, _P]
        l.oracle_lerp.argtypes = [_P, _P, _I, _P, _I, _I, _U64, _D]
        l.oracle_delta_partial.argtypes = [_P, _I, ctypes.POINTER(_P), _I, _I, _I, _U64, _P, _I]
        l.oracle_sgd_apply.argtypes = [_P, _I, _P, _P, _I, _U64, _D, _D, _I]
        l.oracle_max_threads.argtypes = []
        l.oracle_set_threads.argtypes = [_I]
        l.oracle_ref_sdot.argtypes = [_P, _P, ctypes.c_int64, _I]
        l.oracle_ref_sdot.restype = ctypes.c_float
        l.oracle_np_sum_f32.argtypes = [_P, ctypes.c_int64]
        l.oracle_np_sum_f32.restype = ctypes.c_float
        l.oracle_ref_slerp_dot.argtypes = [_P, _P, _I, ctypes.c_int64, _I, ctypes.c_float,
                                           ctypes.POINTER(ctypes.c_float), ctypes.POINTER(ctypes.c_float),
                                           ctypes.POINTER(ctypes.c_float)]
        for f in (l.oracle_outer_step, l.oracle_pair_merge, l.oracle_lerp, l.oracle_max_threads, l.oracle_set_threads,
                  l.oracle_delta_partial, l.oracle_sgd_apply, l.oracle_ref_slerp_dot):
            f.restype = _I
        _lib = l
    return _lib


def _cpu(t: torch.Tensor) -> torch.Tensor:
    assert t.device.type == "cpu" and t.is_contiguous(), "oracle operands: contiguous CPU tensors"
    assert t.dtype in _DT, t.dtype
    return t


def torch_cpu_tail_mask(numels: list[int], vec_elems: int = 32, num_threads: int = 1,
                        grain: int = 32768) -> torch.Tensor:
    """Elements a flat concatenation of tensors (sizes `numels`) sends down torch's scalar
    tail when torch's CPU kernels process each tensor (aten/native/cpu/Loops.h vectorized_loop:
    the last n % Vec::size() elements of every contiguous run; runs are at::parallel_for chunks
    of ceil(numel / min(threads, ceil(numel / grain))) elements). Vec::size() is 32 bf16 on an
    AVX-512 host (16 on AVX2)."""
    mask = torch.zeros(sum(numels), dtype=torch.uint8)
    off = 0
    for n in numels:
        tasks = max(1, min(num_threads, -(-n // grain)))
        chunk = -(-n // tasks) if n else 0
        for b in range(0, n, max(chunk, 1)):
            e = min(n, b + chunk)
            t0 = b + (e - b) // vec_elems * vec_elems
            mask[off + t0:off + e] = 1
        off += n
    return mask


def _tail_ptr(tail):
    if tail is None:
        return 0
    assert tail.dtype == torch.uint8 and tail.is_contiguous()
    return tail.data_ptr()


def outer_step(theta: torch.Tensor, workers: list[torch.Tensor], momentum: torch.Tensor | None,
               has_momentum: bool, lr: float, mu: float, nesterov: bool,
               tail: torch.Tensor | None = None) -> None:
    """EDT_LM/diloco.py:238-289 on flat tensors, in place on theta (and momentum).
    tail: optional torch_cpu_tail_mask() to reproduce torch CPU's bf16 scalar tails."""
    _cpu(theta)
    arr = (_P * len(workers))(*[_cpu(w).data_ptr() for w in workers])
    wdt = _DT[workers[0].dtype]
    assert all(w.numel() == theta.numel() and _DT[w.dtype] == wdt for w in workers)
    mp = 0 if momentum is None else _cpu(momentum).data_ptr()
    rc = lib().oracle_outer_step(theta.data_ptr(), _DT[theta.dtype], arr, wdt, len(workers), mp,
                                 int(has_momentum), theta.numel(), lr, mu, int(nesterov), _tail_ptr(tail))
    assert rc == 0, rc


def delta_partial(theta, workers, k_total, acc, accumulate=False) -> None:
    """Sharded form of the delta accumulate: acc (fp32) (+)= sum over `workers`."""
    arr = (_P * len(workers))(*[_cpu(w).data_ptr() for w in workers])
    assert acc.dtype == torch.float32
    rc = lib().oracle_delta_partial(_cpu(theta).data_ptr(), _DT[theta.dtype], arr, _DT[workers[0].dtype],
                                    len(workers), int(k_total), theta.numel(), _cpu(acc).data_ptr(),
                                    int(accumulate))
    assert rc == 0, rc


def sgd_apply(theta, acc, momentum, has_momentum, lr, mu, nesterov) -> None:
    """Sharded form of the SGD step from an fp32 pseudo-gradient sum."""
    mp = 0 if momentum is None else _cpu(momentum).data_ptr()
    rc = lib().oracle_sgd_apply(_cpu(theta).data_ptr(), _DT[theta.dtype], _cpu(acc).data_ptr(), mp,
                                int(has_momentum), theta.numel(), lr, mu, int(nesterov))
    assert rc == 0, rc


def pair_merge(b1, b2, m1, m2, theta_out, momentum, has_momentum, lr, mu, nesterov, tail=None) -> None:
    """EDT_LM/train/crossover.py:150-230 (b2 None: b1 is the merged base)."""
    wdt = _DT[_cpu(m1).dtype]
    mp = 0 if momentum is None else _cpu(momentum).data_ptr()
    rc = lib().oracle_pair_merge(_cpu(b1).data_ptr(), 0 if b2 is None else _cpu(b2).data_ptr(),
                                 m1.data_ptr(), _cpu(m2).data_ptr(), wdt, _cpu(theta_out).data_ptr(),
                                 _DT[theta_out.dtype], mp, int(has_momentum), theta_out.numel(),
                                 lr, mu, int(nesterov), _tail_ptr(tail))
    assert rc == 0, rc


def lerp(t: float, v0: torch.Tensor, v1: torch.Tensor, compute_dtype=None, out_dtype=None) -> torch.Tensor:
    """(1-t)*v0 + t*v1, three rounded ops in compute_dtype (default: the inputs' dtype)."""
    cdt = compute_dtype or v0.dtype
    out = torch.empty(v0.shape, dtype=out_dtype or cdt)
    rc = lib().oracle_lerp(_cpu(v0).data_ptr(), _cpu(v1).data_ptr(), _DT[v0.dtype], out.data_ptr(),
                           _DT[out.dtype], _DT[cdt], v0.numel(), t)
    assert rc == 0, rc
    return out


def max_threads() -> int:
    return lib().oracle_max_threads()


def set_threads(n: int) -> int:
    """OpenMP team size of the C restatement's loops; returns the size now in effect."""
    return lib().oracle_set_threads(int(n))


# ------------------------------------------------------------------------------------------
# SLERP restated in numpy (EDT_RL/crossover.py:11-81). numpy >= 2 (NEP 50): python floats
# combine with float32 arrays/scalars as float32.

def _unit(v: np.ndarray, eps: float) -> np.ndarray:
    n = np.linalg.norm(v)                 # sqrt(dot(v.ravel(), v.ravel())) in float32
    return v / n if n > eps else v


def slerp_parts(t: float, v0, v1, dot_threshold: float = 0.9995, eps: float = 1e-8):
    """Returns (result float32 ndarray, dot, used_lerp_branch)."""
    a = v0.detach().cpu().float().numpy() if isinstance(v0, torch.Tensor) else np.asarray(v0)
    b = v1.detach().cpu().float().numpy() if isinstance(v1, torch.Tensor) else np.asarray(v1)
    dot = np.sum(_unit(a, eps) * _unit(b, eps))
    if np.abs(dot) > dot_threshold:
        return (1 - t) * a + t * b, dot, True
    th0 = np.arccos(dot)
    th_t = th0 * t
    s0 = np.sin(th0 - th_t) / np.sin(th0)
    s1 = np.sin(th_t) / np.sin(th0)
    return s0 * a + s1 * b, dot, False


def ref_sdot(x: np.ndarray, y: np.ndarray, threads: int = 1) -> np.float32:
    """BLAS sdot as the reference host's numpy runs it (edt_oracle.c: OpenBLAS 0.3.29 SkylakeX)."""
    x = np.ascontiguousarray(x, dtype=np.float32).ravel()
    y = np.ascontiguousarray(y, dtype=np.float32).ravel()
    return np.float32(lib().oracle_ref_sdot(x.ctypes.data, y.ctypes.data, x.size, threads))


def np_sum_f32(a: np.ndarray) -> np.float32:
    """np.sum of a contiguous float32 array (8192-element buffers, pairwise inside), restated."""
    a = np.ascontiguousarray(a, dtype=np.float32).ravel()
    return np.float32(lib().oracle_np_sum_f32(a.ctypes.data, a.size))


def ref_slerp_dot(v0, v1, threads: int = 1, eps: float = 1e-8):
    """(dot, norm0, norm1) of EDT_RL/crossover.py:20-29 from the restatement (no numpy reduction):
    what the reference's own numpy computes on a host with this BLAS model."""
    a, b = _cpu(torch.as_tensor(v0)).reshape(-1), _cpu(torch.as_tensor(v1)).reshape(-1)
    d, n0, n1 = ctypes.c_float(), ctypes.c_float(), ctypes.c_float()
    rc = lib().oracle_ref_slerp_dot(a.data_ptr(), b.data_ptr(), _DT[a.dtype], a.numel(), threads, eps,
                                    ctypes.byref(d), ctypes.byref(n0), ctypes.byref(n1))
    assert rc == 0, rc
    return np.float32(d.value), np.float32(n0.value), np.float32(n1.value)


def slerp_parts_refdot(t: float, v0, v1, threads: int = 1, dot_threshold: float = 0.9995, eps: float = 1e-8):
    """EDT_RL/crossover.py:11-43 with the dot from the pinned BLAS / numpy restatement
    (ref_slerp_dot) instead of this host's live BLAS — the reference as it runs on the pinned
    reference host, whatever BLAS kernel this host's numpy dispatches to: the coefficients and the
    blend are numpy's own float32 ops, as slerp_parts'. Returns (result float32 ndarray, dot,
    used_lerp_branch). On the fixture host it equals slerp_parts bit for bit (tests/test_refdot_cpu.py)."""
    a = v0.detach().cpu().float().numpy() if isinstance(v0, torch.Tensor) else np.asarray(v0, dtype=np.float32)
    b = v1.detach().cpu().float().numpy() if isinstance(v1, torch.Tensor) else np.asarray(v1, dtype=np.float32)
    dot, _, _ = ref_slerp_dot(torch.from_numpy(np.ascontiguousarray(a)), torch.from_numpy(np.ascontiguousarray(b)),
                              threads, eps)
    c0, c1 = slerp_coefficients_at_dot(t, dot, dot_threshold)
    return c0 * a + c1 * b, dot, bool(np.abs(dot) > dot_threshold)


def canonical_chunk_sums(v0, v1, chunks) -> np.ndarray:
    """The product's fp64 chunk sums {v0.v0, v1.v1, v0.v1} [nchunks, 3] in its documented canonical
    order (edt_slerp.hip, "the chunk sums' canonical order") — not the reference's
    order (it sums in fp32 with numpy): this pins that every kernel form computes exactly the
    order the design states. Per chunk [start, start + len): the 8-aligned body in 128 tiles of
    64 lanes x 8 elements, each lane an fp64 FMA chain in element order (a float32 product is exact
    in fp64, so s + x * x here rounds once, as the FMA does); tile 0's lanes then take the head /
    tail elements; the descending xor butterfly (32 .. 1) per tile; the perfect binary tree over the
    128 tile sums, adjacent pairs first."""
    x = _cpu(torch.as_tensor(v0)).reshape(-1).float().numpy().astype(np.float64)
    y = _cpu(torch.as_tensor(v1)).reshape(-1).float().numpy().astype(np.float64)
    chunks = np.asarray(chunks, dtype=np.int64).reshape(-1, 3)
    out = np.zeros((len(chunks), 3))
    lanes = np.arange(64)
    for c, (start, ln, _) in enumerate(chunks):
        end = start + ln
        a, b = (start + 7) // 8 * 8, end // 8 * 8
        P = np.zeros((3, 128, 64))
        if a < b:
            X, Y = np.zeros(128 * 512), np.zeros(128 * 512)
            X[:b - a], Y[:b - a] = x[a:b], y[a:b]
            X, Y = X.reshape(128, 64, 8), Y.reshape(128, 64, 8)
            for e in range(8):
                xe, ye = X[:, :, e], Y[:, :, e]
                P[0] = P[0] + xe * xe
                P[1] = P[1] + ye * ye
                P[2] = P[2] + xe * ye
        h_end = min(a, end)
        t_beg = b if b > a else h_end
        nh, nt = h_end - start, end - t_beg
        for lane in range(nh + nt):
            i = start + lane if lane < nh else t_beg + lane - nh
            P[:, 0, lane] = P[:, 0, lane] + np.array([x[i] * x[i], y[i] * y[i], x[i] * y[i]])
        for o in (32, 16, 8, 4, 2, 1):
            P = P + P[:, :, lanes ^ o]
        T = P[:, :, 0]
        while T.shape[1] > 1:
            T = T[:, 0::2] + T[:, 1::2]
        out[c] = T[:, 0]
    return out


def slerp(t: float, v0, v1, dot_threshold: float = 0.9995, eps: float = 1e-8) -> torch.Tensor:
    res, _, _ = slerp_parts(t, v0, v1, dot_threshold, eps)
    return torch.from_numpy(np.ascontiguousarray(res))


def slerp_coefficients(t: float, v0, v1, dot_threshold: float = 0.9995, eps: float = 1e-8):
    """The (c0, c1) float32 pair the reference's branch multiplies v0, v1 by, and the dot."""
    a = v0.detach().cpu().float().numpy() if isinstance(v0, torch.Tensor) else np.asarray(v0)
    b = v1.detach().cpu().float().numpy() if isinstance(v1, torch.Tensor) else np.asarray(v1)
    dot = np.sum(_unit(a, eps) * _unit(b, eps))
    if np.abs(dot) > dot_threshold:
        return np.float32(1 - t), np.float32(t), dot
    th0 = np.arccos(dot)
    th_t = th0 * t
    return np.sin(th0 - th_t) / np.sin(th0), np.sin(th_t) / np.sin(th0), dot


def slerp_coefficients_at_dot(t: float, dot, dot_threshold: float = 0.9995):
    """The reference's branch and (c0, c1) (EDT_RL/crossover.py:31-43) for a GIVEN fp32 dot: the
    same numpy float32 ops as slerp_coefficients after its dot. Used to measure the formula's own
    conditioning (how far c moves for a dot a few ulps away)."""
    dot = np.float32(dot)
    if np.abs(dot) > dot_threshold:
        return np.float32(1 - t), np.float32(t)
    th0 = np.arccos(dot)
    th_t = th0 * t
    return np.sin(th0 - th_t) / np.sin(th0), np.sin(th_t) / np.sin(th0)


# ---- the reference's CPU loop as it runs (timing baseline, not a checker) ---------------------

def torch_loop_outer_step(base_params: list[torch.Tensor], worker_params: list[list[torch.Tensor]],
                          optimizer: torch.optim.Optimizer | None, lr: float, mu: float, nesterov: bool):
    """The DiLoCo outer step the way EDT_LM/diloco.py:238-289 executes it on the master's CPU: per
    parameter tensor, a running sum of (trained - base) / num_models built with torch ops (one
    temporary per op), `p.grad = -sum`, then torch.optim.SGD (single-tensor CPU path). Restated
    here so bench.py can time the reference's own cost profile on the GPU box's host, where the
    reference's files are not available. Returns the optimizer (carried across calls)."""
    K = len(worker_params)
    for i, p in enumerate(base_params):
        acc = torch.zeros_like(p)
        for k in range(K):
            acc += (worker_params[k][i] - p) / K
        p.grad = -acc
    if optimizer is None:
        optimizer = torch.optim.SGD(base_params, lr=lr, momentum=mu, nesterov=nesterov)
    optimizer.step()
    optimizer.zero_grad()
    return optimizer
