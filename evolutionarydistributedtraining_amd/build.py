"""Build the in-tree HIP library `libedt_sync.so` for gfx950 (hipcc cross-compiles without a GPU)."""
from __future__ import annotations

import os
import shutil
import subprocess

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(PKG_DIR)
CSRC = os.path.join(PKG_DIR, "csrc")
# one shared object from four translation units (DiLoCo, pair merge + lerp, SLERP, ABI misc)
SOURCES = [os.path.join(CSRC, f) for f in ("edt_outer.hip", "edt_merge.hip", "edt_slerp.hip", "edt_abi.hip")]
HEADER = os.path.join(ROOT, "include", "edt_sync.h")
DEPS = SOURCES + [HEADER, os.path.join(CSRC, "edt_common.h")]
OUT = os.path.join(PKG_DIR, "libedt_sync.so")

# -ffp-contract=off: the kernels reproduce torch's rounding op by op; the only FMAs are the
# explicit ones that restate torch's add(..., alpha=).
HIPCC_FLAGS = ["--offload-arch=gfx950", "-O3", "-std=c++17", "-ffp-contract=off", "-fPIC", "-shared",
               "-Wall", "-Wno-unused-function"]


def hipcc() -> str:
    for c in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if c and os.path.exists(c):
            return c
    raise RuntimeError("hipcc not found (ROCm is required to build the gfx950 kernels)")


def needs_build(out: str = OUT) -> bool:
    if not os.path.exists(out):
        return True
    t = os.path.getmtime(out)
    return any(os.path.getmtime(s) > t for s in DEPS)


def build_library(force: bool = False, extra_flags: list[str] | None = None, out: str = OUT) -> str:
    if force or needs_build(out):
        cmd = [hipcc(), *HIPCC_FLAGS, *(extra_flags or []), "-I", os.path.dirname(HEADER), "-I", CSRC,
               *SOURCES, "-o", out + ".tmp"]
        subprocess.run(cmd, check=True)
        os.replace(out + ".tmp", out)
    return out


if __name__ == "__main__":
    print(build_library(force=True))
