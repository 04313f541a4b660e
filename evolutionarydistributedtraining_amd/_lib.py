"""ctypes binding of `libedt_sync.so` (the C ABI in include/edt_sync.h).

The library is built in-tree by `evolutionarydistributedtraining_amd.build.build_library()` (or
`__graft_entry__.build()`). There is no fallback: if the shared object is missing or a GPU is
not available, every operator raises. Torch is imported first so that the HIP runtime torch
ships (SONAME libamdhip64.so.7) is the one the library binds to.
"""
from __future__ import annotations

import ctypes
import os

import torch

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(PKG_DIR, "libedt_sync.so")

EDT_F32 = 0
EDT_BF16 = 1
EDT_MAX_WORKERS = 64
EDT_ABI_VERSION = 6         # include/edt_sync.h: the revision these signatures and workspace sizes follow

_DT = {torch.float32: EDT_F32, torch.bfloat16: EDT_BF16}

# (name, restype, argtypes) for every symbol declared in include/edt_sync.h
_P = ctypes.c_void_p
_U64 = ctypes.c_uint64
_I = ctypes.c_int
_D = ctypes.c_double
SIGNATURES = [
    ("edt_outer_step", _I, [_P, _I, ctypes.POINTER(_P), _I, _I, _P, _I, _U64, _D, _D, _I, _P]),
    ("edt_outer_step_bcast", _I, [_P, _I, ctypes.POINTER(_P), _I, _I, _P, _I, _U64, _D, _D, _I,
                                  ctypes.POINTER(_P), _I, _P]),
    ("edt_outer_step_tail", _I, [_P, _I, ctypes.POINTER(_P), _I, _I, _P, _I, _U64, _D, _D, _I, _P, _P]),
    ("edt_pair_merge_tail", _I, [_P, _P, _P, _P, _I, _P, _I, _P, _P, _I, _U64, _D, _D, _I, _P, _P]),
    ("edt_outer_step_ws", _I, [_P, _I, ctypes.POINTER(_P), _I, _I, _P, _I, _U64, _D, _D, _I, _P, _P]),
    ("edt_outer_list_workspace_bytes", _U64, [_I, _I]),
    ("edt_outer_step_list", _I, [ctypes.POINTER(_P), _I, ctypes.POINTER(_P), _I, _I, ctypes.POINTER(_P), _I,
                                 ctypes.POINTER(_U64), _I, _D, _D, _I, _P, _U64, _P]),
    ("edt_outer_step_list_tail", _I, [ctypes.POINTER(_P), _I, ctypes.POINTER(_P), _I, _I, ctypes.POINTER(_P), _I,
                                      ctypes.POINTER(_U64), _I, _D, _D, _I, _P, ctypes.POINTER(_U64), _P, _U64, _P]),
    ("edt_delta_partial", _I, [_P, _I, ctypes.POINTER(_P), _I, _I, _I, _U64, _P, _I, _P]),
    ("edt_sgd_apply", _I, [_P, _I, _P, _P, _I, _U64, _D, _D, _I, _P]),
    ("edt_sgd_apply_sum", _I, [_P, _I, ctypes.POINTER(_P), _I, _P, _I, _U64, _D, _D, _I, _P]),
    ("edt_pair_merge", _I, [_P, _P, _P, _P, _I, _P, _I, _P, _I, _U64, _D, _D, _I, _P]),
    ("edt_pair_merge_to", _I, [_P, _P, _P, _P, _I, _P, _I, _P, _P, _I, _U64, _D, _D, _I, _P]),
    ("edt_pair_merge_population", _I, [ctypes.POINTER(_P), ctypes.POINTER(_P), ctypes.POINTER(_P),
                                       ctypes.POINTER(_P), _I, ctypes.POINTER(_P), _I, ctypes.POINTER(_P),
                                       ctypes.POINTER(_P), ctypes.POINTER(ctypes.c_int32), _I, _U64, _D, _D, _I,
                                       _P]),
    ("edt_lerp", _I, [_P, _P, _I, _P, _I, _I, _U64, _D, _P]),
    ("edt_slerp_make_chunks", ctypes.c_int64,
     [ctypes.POINTER(_U64), _I, ctypes.c_uint32, ctypes.POINTER(_U64), ctypes.c_int64,
      ctypes.POINTER(ctypes.c_int32)]),
    ("edt_slerp_stats", _I, [_P, _P, _I, _P, ctypes.c_int64, _P, _P]),
    ("edt_slerp_coef", _I, [_P, _P, _I, _P, _D, _D, _P, _P, _P]),
    ("edt_slerp_blend", _I, [_P, _P, _I, _P, _I, _P, ctypes.c_int64, _P, _P]),
    ("edt_slerp_merge", _I, [_P, _P, _I, _P, _I, _P, ctypes.c_int64, _P, _I, _P, _D, _D, _P, _P, _P, _P]),
    ("edt_slerp_merge_speculative", _I, [_P, _P, _I, _P, _I, _P, ctypes.c_int64, _P, _I, _P, _D, _D, _P, _P, _P,
                                         _P, _U64, _P]),
    ("edt_slerp_merge_list", _I, [ctypes.POINTER(_P), ctypes.POINTER(_P), _I, ctypes.POINTER(_P), _I, _P,
                                  ctypes.c_int64, _P, _I, _P, _D, _D, _P, _P, _P, _P, _U64, _P]),
    ("edt_slerp_merge_list_speculative", _I, [ctypes.POINTER(_P), ctypes.POINTER(_P), _I, ctypes.POINTER(_P), _I,
                                              _P, _P, ctypes.c_int64, _P, _I, _P, _D, _D, _P, _P, _P, _P, _P, _U64,
                                              _P]),
    ("edt_slerp_seg_table", _I, [ctypes.POINTER(_P), ctypes.POINTER(_P), ctypes.POINTER(_P), _I, _P, _I, _I, _I, _P]),
    ("edt_slerp_stats_table", _I, [_P, _I, _P, ctypes.c_int64, _P, _P]),
    ("edt_slerp_blend_table", _I, [_P, _I, _I, _P, ctypes.c_int64, _P, _P, _P]),
    ("edt_slerp_merge_table", _I, [_P, _I, _I, _P, ctypes.c_int64, _P, _I, _P, _D, _D, _P, _P, _P, _P]),
    ("edt_slerp_merge_table_speculative", _I, [_P, _I, _I, _P, ctypes.c_int64, _P, _I, _P, _D, _D, _P, _P, _P, _P,
                                               _P]),
    ("edt_slerp_blend_segments", _I, [_P, _P, _I, _P, _I, _P, ctypes.c_int64, _P, _P, _P]),
    ("edt_slerp_refdot_table", _I, [_P, _I, _P, ctypes.c_int64, _P, _I, ctypes.c_uint32, _P, _I, _D, _P, _P, _U64,
                                    _P]),
    ("edt_slerp_sums_doubles", _U64, [_I, ctypes.c_int64]),
    ("edt_slerp_refdot_workspace_bytes", _U64, [_I, ctypes.c_int64, ctypes.c_uint32, _I]),
    ("edt_slerp_refdot_flags", _I, [_P, _I, _D, _D, _P, _P]),
    ("edt_slerp_refdot", _I, [_P, _P, _I, _P, ctypes.c_int64, _P, _I, ctypes.c_uint32, _P, _I, _D, _P, _P, _U64, _P]),
    ("edt_slerp_refdot_coef", _I, [_P, _P, _I, _P, _D, _P, _P, _P]),
    ("edt_slerp_population_gram_doubles", _U64, [_I, ctypes.c_int64]),
    ("edt_slerp_population_speculative_doubles", _U64, [_I, ctypes.c_int64]),
    ("edt_slerp_population", _I, [ctypes.POINTER(_P), _I, _I, ctypes.POINTER(ctypes.c_int32), _I,
                                  ctypes.POINTER(_P), _I, _P, ctypes.c_int64, _P, _I, _P, _D, _D, _P, _P, _P,
                                  _P]),
    ("edt_slerp_population_speculative", _I, [ctypes.POINTER(_P), _I, _I, ctypes.POINTER(ctypes.c_int32), _I,
                                              ctypes.POINTER(_P), _I, _P, ctypes.c_int64, _P, _I, _P, _D, _D, _P,
                                              _P, _P, _P, _U64, _P]),
    ("edt_slerp_population_layout", _I, [ctypes.POINTER(ctypes.c_int32), _I, _I, _I, ctypes.c_char_p, _I]),
    ("edt_slerp_needed_table", _I, [ctypes.POINTER(ctypes.c_int32), _I, _I, ctypes.c_int64, ctypes.POINTER(_U64),
                                    ctypes.POINTER(ctypes.c_int32), ctypes.POINTER(ctypes.c_int32),
                                    ctypes.POINTER(ctypes.c_int32), ctypes.POINTER(_U64), ctypes.POINTER(_U64)]),
    ("edt_slerp_needed_sums", _I, [ctypes.POINTER(_P), _I, _I, ctypes.POINTER(ctypes.c_int32), _I, _P, ctypes.c_int64,
                                   ctypes.c_int64, ctypes.c_int64, _P, _P, _U64, _P]),
    ("edt_slerp_needed_coef", _I, [_P, ctypes.c_int64, ctypes.POINTER(ctypes.c_int32), _I, _I, _P, _I, _P, _D, _D,
                                   _P, _P, _P]),
    ("edt_slerp_blend_children", _I, [ctypes.POINTER(_P), _I, _I, ctypes.POINTER(ctypes.c_int32), _I,
                                      ctypes.POINTER(_P), _I, _P, ctypes.c_int64, _P, _I, _P]),
    ("edt_probe_stream", _I, [_P, _I, ctypes.POINTER(_P), _I, _I, _P, _U64, _P]),
    ("edt_last_error", ctypes.c_char_p, []),
    ("edt_version", ctypes.c_char_p, []),
    ("edt_abi_version", _I, []),
    ("edt_outer_step_bytes_per_elem", _I, [_I, _I, _I, _I]),
]

_lib = None


class EdtError(RuntimeError):
    """A C-ABI call returned a negative status (message from edt_last_error())."""


_sha_cache: dict = {}


def library_sha256(path: str = LIB_PATH) -> str | None:
    """sha256 of the library file: the build stamp that ties a profile (profiles/pmc_traffic.json)
    to the exact kernels it was measured on."""
    if path not in _sha_cache:
        import hashlib
        try:
            with open(path, "rb") as f:
                _sha_cache[path] = hashlib.sha256(f.read()).hexdigest()
        except OSError:
            return None
    return _sha_cache[path]


def load_library(path: str = LIB_PATH) -> ctypes.CDLL:
    """Load and bind the shared object (no GPU needed). Raises if it is missing."""
    global _lib
    if _lib is not None and path == LIB_PATH:
        return _lib
    if not os.path.exists(path):
        raise EdtError(
            f"{path} is missing: build it with `python -c 'import __graft_entry__ as g; g.build()'` "
            "(hipcc --offload-arch=gfx950). There is no CPU fallback.")
    lib = ctypes.CDLL(path, mode=ctypes.RTLD_GLOBAL)
    ver = getattr(lib, "edt_abi_version", None)
    if ver is None:
        raise EdtError(f"{path} predates the versioned ABI: rebuild it (this binding follows ABI {EDT_ABI_VERSION})")
    ver.restype, ver.argtypes = _I, []
    if ver() != EDT_ABI_VERSION:
        raise EdtError(f"{path} implements ABI {ver()}, this binding follows ABI {EDT_ABI_VERSION}: rebuild it")
    for name, res, args in SIGNATURES:
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    if path == LIB_PATH:
        _lib = lib
    return lib


def lib() -> ctypes.CDLL:
    """The bound library, for device work: also insists on a visible GPU."""
    l = load_library()
    if not torch.cuda.is_available():
        raise EdtError("no HIP device visible: the outer-loop sync kernels run on MI355X only")
    return l


def check(rc: int, what: str) -> None:
    if rc != 0:
        msg = load_library().edt_last_error().decode(errors="replace")
        raise EdtError(f"{what} failed ({rc}): {msg}")


def dtype_code(t: torch.Tensor | torch.dtype) -> int:
    dt = t if isinstance(t, torch.dtype) else t.dtype
    if dt not in _DT:
        raise EdtError(f"unsupported dtype {dt}: the kernels take float32 or bfloat16")
    return _DT[dt]


def stream_ptr(device: torch.device | None = None) -> ctypes.c_void_p:
    return ctypes.c_void_p(torch.cuda.current_stream(device).cuda_stream)


def ptr(t: torch.Tensor | None) -> ctypes.c_void_p:
    return ctypes.c_void_p(0 if t is None else t.data_ptr())


def ptr_array(tensors) -> ctypes.Array:
    arr = (ctypes.c_void_p * max(1, len(tensors)))()
    for i, t in enumerate(tensors):
        arr[i] = t.data_ptr()
    return arr


def require_device(*tensors: torch.Tensor) -> torch.device:
    """All tensors on one HIP device and contiguous; returns that device."""
    dev = None
    for t in tensors:
        if t is None:
            continue
        if not t.is_cuda:
            raise EdtError("outer-loop sync operands must be device-resident (HBM) tensors")
        if not t.is_contiguous():
            raise EdtError("outer-loop sync operands must be contiguous")
        if dev is None:
            dev = t.device
        elif t.device != dev:
            raise EdtError(f"operands on different devices: {dev} vs {t.device}")
    return dev
