"""ctypes binding of libedt_comm.so (include/edt_comm.h): RCCL over xGMI and the bucketed DiLoCo
reduce schedule behind the C ABI, for hosts without torch.distributed (a Go / Java / C master
driving one process per GPU). The Python package's own multi-GPU path is distributed.py
(torch.distributed "nccl", the same librccl); this module is the C boundary's binding and is what
the GPU tests drive. No CPU fallback: loading needs librccl, every call a HIP device.
"""
from __future__ import annotations

import ctypes
import os

import torch

from . import _lib as L

_PATH = os.path.join(os.path.dirname(os.path.abspath(__file__)), "libedt_comm.so")
_LIB = None

_P, _I, _U64, _D = ctypes.c_void_p, ctypes.c_int, ctypes.c_uint64, ctypes.c_double
SIGNATURES = [
    ("edt_comm_id_bytes", _U64, []),
    ("edt_comm_unique_id", _I, [_P]),
    ("edt_comm_init", _I, [ctypes.POINTER(_P), _P, _I, _I]),
    ("edt_comm_destroy", _I, [_P]),
    ("edt_comm_rank", _I, [_P]),
    ("edt_comm_size", _I, [_P]),
    ("edt_comm_reduce_scatter_f32", _I, [_P, _P, _P, _U64, _P]),
    ("edt_comm_all_gather", _I, [_P, _P, _P, _U64, _I, _P]),
    ("edt_comm_all_to_all", _I, [_P, _P, _P, _U64, _I, _P]),
    ("edt_comm_exchange", _I, [_P, ctypes.POINTER(ctypes.c_int32), ctypes.POINTER(ctypes.c_int32),
                               ctypes.POINTER(_P), ctypes.POINTER(_P), ctypes.POINTER(_U64), _I, _P]),
    ("edt_outer_step_sharded", _I, [_P, _P, _I, ctypes.POINTER(_P), _I, _I, _P, _I, _U64, _U64, _D, _D, _I,
                                    _P, _P]),
    ("edt_outer_step_sharded_ordered", _I, [_P, _P, _I, ctypes.POINTER(_P), _I, _I, _P, _I, _U64, _U64, _D, _D,
                                            _I, _P, _P, _P]),
    ("edt_outer_step_sharded_exact", _I, [_P, _P, _I, ctypes.POINTER(_P), _I, _I, _P, _I, _U64, _U64, _D, _D,
                                          _I, ctypes.POINTER(_P), _P]),
    ("edt_comm_abort", _I, [_P]),
    ("edt_comm_poll", _I, [_P]),
    ("edt_comm_wait", _I, [_P, _P, _D]),
    ("edt_comm_set_timeout", _I, [_P, _D]),
    ("edt_comm_last_error", ctypes.c_char_p, []),
]

ERR_ABORTED, ERR_TIMEOUT = -4, -5


def load_comm_library():
    """libedt_comm.so with every entry point typed (libedt_sync.so is loaded first: the comm
    library links it and resolves to the same copy)."""
    global _LIB
    if _LIB is None:
        L.load_library()
        if not os.path.exists(_PATH):
            raise L.EdtError(f"{_PATH} is missing: build it (python -c 'import __graft_entry__ as g; g.build()')")
        lib = ctypes.CDLL(_PATH)
        for name, res, args in SIGNATURES:
            f = getattr(lib, name)
            f.restype, f.argtypes = res, args
        _LIB = lib
    return _LIB


def _check(rc: int, what: str) -> None:
    if rc != 0:
        raise L.EdtError(f"{what} failed ({rc}): {load_comm_library().edt_comm_last_error().decode()}")


class Comm:
    """One rank's RCCL communicator through the C ABI."""

    @staticmethod
    def unique_id() -> bytes:
        lib = load_comm_library()
        buf = ctypes.create_string_buffer(int(lib.edt_comm_id_bytes()))
        _check(lib.edt_comm_unique_id(buf), "edt_comm_unique_id")
        return buf.raw

    def __init__(self, uid: bytes, nranks: int, rank: int):
        lib = load_comm_library()
        self._h = _P()
        _check(lib.edt_comm_init(ctypes.byref(self._h), ctypes.create_string_buffer(uid, len(uid)), nranks, rank),
               "edt_comm_init")
        self.rank, self.size = lib.edt_comm_rank(self._h), lib.edt_comm_size(self._h)

    def close(self) -> None:
        if self._h:
            _check(load_comm_library().edt_comm_destroy(self._h), "edt_comm_destroy")
            self._h = _P()

    def abort(self) -> None:
        """ncclCommAbort: outstanding collectives end; later calls fail with EDT_COMM_ERR_ABORTED."""
        _check(load_comm_library().edt_comm_abort(self._h), "edt_comm_abort")

    def poll(self) -> None:
        """Raise EdtError if the communicator was aborted or holds an asynchronous RCCL error."""
        _check(load_comm_library().edt_comm_poll(self._h), "edt_comm_poll")

    def wait(self, device=None, timeout_s: float = 0.0) -> None:
        """Host wait for the work on the current stream and the communicator's own; past
        timeout_s the communicator is aborted and EdtError raised (EDT_COMM_ERR_TIMEOUT)."""
        dev = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
        _check(load_comm_library().edt_comm_wait(self._h, L.stream_ptr(dev), float(timeout_s)), "edt_comm_wait")

    def set_timeout(self, seconds: float) -> None:
        """> 0: outer_step_sharded waits for its work and fails after `seconds` (edt_comm_set_timeout)."""
        _check(load_comm_library().edt_comm_set_timeout(self._h, float(seconds)), "edt_comm_set_timeout")

    def _stream(self, t: torch.Tensor):
        return L.stream_ptr(t.device)

    def reduce_scatter_f32(self, send: torch.Tensor, recv: torch.Tensor) -> None:
        if send.dtype != torch.float32 or recv.dtype != torch.float32 or send.numel() != recv.numel() * self.size:
            raise L.EdtError("reduce_scatter_f32: fp32 send of size x recv")
        L.require_device(send, recv)
        _check(load_comm_library().edt_comm_reduce_scatter_f32(self._h, L.ptr(send), L.ptr(recv), recv.numel(),
                                                              self._stream(send)), "edt_comm_reduce_scatter_f32")

    def all_gather(self, send: torch.Tensor, recv: torch.Tensor) -> None:
        if send.dtype != recv.dtype or recv.numel() != send.numel() * self.size:
            raise L.EdtError("all_gather: recv holds size x send of one dtype")
        L.require_device(send, recv)
        _check(load_comm_library().edt_comm_all_gather(self._h, L.ptr(send), L.ptr(recv), send.numel(),
                                                      L.dtype_code(send), self._stream(send)), "edt_comm_all_gather")

    def all_to_all(self, send: torch.Tensor, recv: torch.Tensor) -> None:
        if send.dtype != recv.dtype or send.numel() != recv.numel() or send.numel() % self.size:
            raise L.EdtError("all_to_all: equal buffers of one dtype, a multiple of the rank count")
        L.require_device(send, recv)
        _check(load_comm_library().edt_comm_all_to_all(self._h, L.ptr(send), L.ptr(recv), send.numel() // self.size,
                                                      L.dtype_code(send), self._stream(send)), "edt_comm_all_to_all")

    def exchange(self, ops) -> None:
        """ops: (send_to, send_tensor, recv_from, recv_tensor) tuples; -1 / None for no side."""
        n = len(ops)
        st = (ctypes.c_int32 * max(1, n))(*[o[0] for o in ops])
        rf = (ctypes.c_int32 * max(1, n))(*[o[2] for o in ops])
        sb = (_P * max(1, n))(*[L.ptr(o[1]) if o[1] is not None else None for o in ops])
        rb = (_P * max(1, n))(*[L.ptr(o[3]) if o[3] is not None else None for o in ops])
        nb = []
        for to, s, frm, r in ops:
            ss = s.numel() * s.element_size() if s is not None else None
            rs = r.numel() * r.element_size() if r is not None else None
            if ss is not None and rs is not None and ss != rs:
                raise L.EdtError("an op's send and receive buffers must have the same size")
            nb.append(ss if ss is not None else rs)
        by = (_U64 * max(1, n))(*nb)
        dev = next(t for o in ops for t in (o[1], o[3]) if t is not None).device if ops else torch.device("cuda")
        _check(load_comm_library().edt_comm_exchange(self._h, st, rf, sb, rb, by, n, L.stream_ptr(dev)),
               "edt_comm_exchange")

    def outer_step_sharded(self, theta: torch.Tensor, workers: list[torch.Tensor], momentum_shard: torch.Tensor | None,
                           has_momentum: bool, lr: float, momentum_coef: float, nesterov: bool,
                           acc: torch.Tensor, bucket_elems: int = 1 << 26) -> None:
        """edt_outer_step_sharded: theta and workers padded flat (n_pad a multiple of size x 64),
        momentum_shard n_pad / size elements of theta's dtype, acc an n_pad fp32 workspace."""
        n = theta.numel()
        L.require_device(theta, acc, *workers, *([momentum_shard] if momentum_shard is not None else []))
        if any(w.numel() != n or w.dtype != workers[0].dtype for w in workers) or acc.numel() != n \
                or acc.dtype != torch.float32:
            raise L.EdtError("workers / acc must match the padded theta")
        _check(load_comm_library().edt_outer_step_sharded(
            self._h, L.ptr(theta), L.dtype_code(theta), L.ptr_array(workers), L.dtype_code(workers[0]), len(workers),
            L.ptr(momentum_shard) if momentum_shard is not None else None, int(has_momentum), n, bucket_elems,
            float(lr), float(momentum_coef), int(nesterov), L.ptr(acc), self._stream(theta)), "edt_outer_step_sharded")

    def outer_step_sharded_ordered(self, theta: torch.Tensor, workers: list[torch.Tensor],
                                   momentum_shard: torch.Tensor | None, has_momentum: bool, lr: float,
                                   momentum_coef: float, nesterov: bool, acc: torch.Tensor, recv: torch.Tensor,
                                   bucket_elems: int = 1 << 26) -> None:
        """edt_outer_step_sharded_ordered (the reduce_ordered schedule): as outer_step_sharded,
        plus `recv`, a second n_pad fp32 workspace the partials' all-to-all lands in."""
        n = theta.numel()
        L.require_device(theta, acc, recv, *workers, *([momentum_shard] if momentum_shard is not None else []))
        if any(w.numel() != n or w.dtype != workers[0].dtype for w in workers) or acc.numel() != n \
                or acc.dtype != torch.float32 or recv.numel() != n or recv.dtype != torch.float32:
            raise L.EdtError("workers / acc / recv must match the padded theta")
        _check(load_comm_library().edt_outer_step_sharded_ordered(
            self._h, L.ptr(theta), L.dtype_code(theta), L.ptr_array(workers), L.dtype_code(workers[0]), len(workers),
            L.ptr(momentum_shard) if momentum_shard is not None else None, int(has_momentum), n, bucket_elems,
            float(lr), float(momentum_coef), int(nesterov), L.ptr(acc), L.ptr(recv), self._stream(theta)),
            "edt_outer_step_sharded_ordered")

    def outer_step_sharded_exact(self, theta: torch.Tensor, workers: list[torch.Tensor],
                                 momentum_shard: torch.Tensor | None, has_momentum: bool, lr: float,
                                 momentum_coef: float, nesterov: bool, recv: list[torch.Tensor],
                                 bucket_elems: int = 1 << 26) -> None:
        """edt_outer_step_sharded_exact (the exact schedule, theta broadcast): recv holds one
        padded buffer of the workers' dtype per local worker, where their all-to-alls land."""
        n = theta.numel()
        L.require_device(theta, *workers, *recv, *([momentum_shard] if momentum_shard is not None else []))
        if len(recv) != len(workers) or any(t.numel() != n or t.dtype != workers[0].dtype for t in workers + recv):
            raise L.EdtError("workers / recv must match the padded theta, one receive buffer per worker")
        _check(load_comm_library().edt_outer_step_sharded_exact(
            self._h, L.ptr(theta), L.dtype_code(theta), L.ptr_array(workers), L.dtype_code(workers[0]), len(workers),
            L.ptr(momentum_shard) if momentum_shard is not None else None, int(has_momentum), n, bucket_elems,
            float(lr), float(momentum_coef), int(nesterov), L.ptr_array(recv), self._stream(theta)),
            "edt_outer_step_sharded_exact")
