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


# Per-translation-unit device flags. edt_slerp.hip: uniform (scalar) control flow is left
# unstructured, so a switch on a kernel argument — the needed-sums pass picks each dot slot's
# member pair with one (edt_slerp.hip, need_dot) — is a plain binary tree of scalar compares and
# branches instead of the structurizer's flag-variable chain (~40 % fewer instructions in that
# pass; divergent regions are structured as before).
TU_FLAGS = {"edt_slerp.hip": ["-mllvm", "-structurizecfg-skip-uniform-regions=true"]}


def build_library(force: bool = False, extra_flags: list[str] | None = None, out: str = OUT,
                  tu_extra: dict | None = None) -> str:
    """One object per translation unit, compiled in parallel (build/obj), then linked. extra_flags:
    added to every unit (variant builds: -D tunables); tu_extra: {file name: flags} for one unit."""
    if force or needs_build(out):
        from concurrent.futures import ThreadPoolExecutor
        objdir = os.path.join(ROOT, "build", "obj", os.path.basename(out))
        os.makedirs(objdir, exist_ok=True)
        flags = [f for f in HIPCC_FLAGS if f != "-shared"]

        def compile_one(src):
            obj = os.path.join(objdir, os.path.basename(src) + ".o")
            cmd = [hipcc(), *flags, *TU_FLAGS.get(os.path.basename(src), []), *(extra_flags or []),
                   *(tu_extra or {}).get(os.path.basename(src), []),
                   "-I", os.path.dirname(HEADER), "-I", CSRC, "-c", src, "-o", obj]
            subprocess.run(cmd, check=True)
            return obj

        with ThreadPoolExecutor(max_workers=len(SOURCES)) as pool:
            objs = list(pool.map(compile_one, SOURCES))
        subprocess.run([hipcc(), "--offload-arch=gfx950", "-shared", "-fPIC", *objs, "-o", out + ".tmp"], check=True)
        os.replace(out + ".tmp", out)
    return out


COMM_SOURCE = os.path.join(CSRC, "edt_comm.cpp")
COMM_HEADER = os.path.join(ROOT, "include", "edt_comm.h")
COMM_OUT = os.path.join(PKG_DIR, "libedt_comm.so")


def build_comm_library(force: bool = False) -> str:
    """libedt_comm.so (include/edt_comm.h): RCCL behind the C ABI, host code only, linked against
    libedt_sync.so (its kernels) and librccl; runpath $ORIGIN so the two travel together."""
    sync = build_library()
    deps = [COMM_SOURCE, COMM_HEADER, HEADER, sync]
    if force or not os.path.exists(COMM_OUT) or any(os.path.getmtime(d) > os.path.getmtime(COMM_OUT) for d in deps):
        rocm = os.path.dirname(os.path.dirname(os.path.realpath(hipcc())))
        cmd = [hipcc(), "-O2", "-std=c++17", "-fPIC", "-shared", "-Wall", "-I", os.path.dirname(HEADER),
               COMM_SOURCE, "-o", COMM_OUT + ".tmp", "-L", PKG_DIR, "-ledt_sync", "-L", os.path.join(rocm, "lib"),
               "-lrccl", "-Wl,-rpath,$ORIGIN", "-Wl,-rpath," + os.path.join(rocm, "lib")]
        subprocess.run(cmd, check=True)
        os.replace(COMM_OUT + ".tmp", COMM_OUT)
    return COMM_OUT


if __name__ == "__main__":
    print(build_library(force=True))
    print(build_comm_library(force=True))
