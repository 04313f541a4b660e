"""roctx ranges around the shim's phases (SURVEY.md §5 tracing): visible to `rocprofv3
--marker-trace` beside the kernels, free otherwise (roctx calls are no-ops without a tool). The
reference's only tracing is tqdm progress bars (EDT_LM/diloco.py:97, EDT_EVOMERGE/train/
crossover.py:121). EDT_ROCTX=0 disables them; a missing librocprofiler-sdk-roctx makes them no-ops."""
from __future__ import annotations

import contextlib
import ctypes
import os

_lib = None
_tried = False


def _roctx():
    global _lib, _tried
    if not _tried:
        _tried = True
        if os.environ.get("EDT_ROCTX", "1") != "0":
            for name in ("librocprofiler-sdk-roctx.so.1", "librocprofiler-sdk-roctx.so", "libroctx64.so.4",
                         "libroctx64.so"):
                for d in ("", "/opt/rocm/lib/"):
                    try:
                        lib = ctypes.CDLL(d + name)
                    except OSError:
                        continue
                    lib.roctxRangePushA.argtypes = [ctypes.c_char_p]
                    lib.roctxRangePushA.restype = ctypes.c_int
                    lib.roctxRangePop.argtypes = []
                    lib.roctxRangePop.restype = ctypes.c_int
                    _lib = lib
                    return _lib
    return _lib


@contextlib.contextmanager
def trange(name: str):
    """`with trange("edt/outer_step"): ...` — one roctx range (host-side push/pop)."""
    lib = _roctx()
    if lib is None:
        yield
        return
    lib.roctxRangePushA(name.encode())
    try:
        yield
    finally:
        lib.roctxRangePop()


def traced(name: str):
    """Decorator form of trange."""
    def deco(fn):
        def wrapper(*a, **kw):
            with trange(name):
                return fn(*a, **kw)
        wrapper.__name__, wrapper.__doc__, wrapper.__wrapped__ = fn.__name__, fn.__doc__, fn
        return wrapper
    return deco


def available() -> bool:
    return _roctx() is not None
