"""Build the in-tree HIP library `libedt_sync.so` for gfx950 (hipcc cross-compiles without a GPU).

The build is source-determined: the same sources and flags give the same bytes at any checkout
path. Each translation unit gets a fixed CUID (`-cuid=<sha of the unit's source>`: hipcc's default
hashes the build path into the `__hip_cuid_*` symbol names) and every path is remapped to `.`
(`-ffile-prefix-map`), so the library's sha256 — the stamp `profiles/pmc_traffic.json` entries
carry — identifies the source, not the directory it was built in (tests/test_build_repro.py)."""
from __future__ import annotations

import hashlib
import json
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

ARCH = "gfx950"
# -ffp-contract=off: the kernels reproduce torch's rounding op by op; the only FMAs are the
# explicit ones that restate torch's add(..., alpha=).
HIPCC_FLAGS = [f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-ffp-contract=off", "-fPIC", "-shared",
               "-Wall", "-Wno-unused-function"]

# Per-translation-unit device flags. edt_slerp.hip: uniform (scalar) control flow is left
# unstructured, so a switch on a kernel argument — the needed-sums pass picks each dot slot's
# member pair with one (edt_slerp.hip, need_dot) — is a plain binary tree of scalar compares and
# branches instead of the structurizer's flag-variable chain (~40 % fewer instructions in that
# pass; divergent regions are structured as before).
TU_FLAGS = {"edt_slerp.hip": ["-mllvm", "-structurizecfg-skip-uniform-regions=true"]}


def hipcc() -> str:
    for c in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if c and os.path.exists(c):
            return c
    raise RuntimeError("hipcc not found (ROCm is required to build the gfx950 kernels)")


def _arch_flags() -> list[str]:
    return [f for f in HIPCC_FLAGS if f.startswith("--offload-arch=")]


def _file_sha(path: str) -> str:
    with open(path, "rb") as f:
        return hashlib.sha256(f.read()).hexdigest()


def _flags_key(out: str, extra_flags, tu_extra) -> str:
    """What, besides the sources, decides the library's bytes — the compiler flags (common, per
    unit, variant) — and the output path, so two builds never share an object directory. Stored
    beside the library; a change forces a rebuild."""
    rec = {"hipcc": HIPCC_FLAGS, "tu": TU_FLAGS, "extra": list(extra_flags or []),
           "tu_extra": {k: list(v) for k, v in sorted((tu_extra or {}).items())}, "out": os.path.abspath(out)}
    return hashlib.sha256(json.dumps(rec, sort_keys=True).encode()).hexdigest()[:16]


def _stamp_path(out: str) -> str:
    return out + ".flags"


def needs_build(out: str = OUT, extra_flags=None, tu_extra=None) -> bool:
    if not os.path.exists(out):
        return True
    t = os.path.getmtime(out)
    if any(os.path.getmtime(s) > t for s in DEPS):
        return True
    try:
        with open(_stamp_path(out)) as f:
            return f.read().strip() != _flags_key(out, extra_flags, tu_extra)
    except OSError:
        return True


def unit_command(src: str, obj: str, extra_flags=None, tu_extra=None) -> list[str]:
    """The hipcc line of one translation unit: fixed CUID from the source's sha256, every path
    under the checkout (and the object's directory) mapped to '.'."""
    name = os.path.basename(src)
    flags = [f for f in HIPCC_FLAGS if f != "-shared"]
    return [hipcc(), *flags, *TU_FLAGS.get(name, []), *(extra_flags or []), *(tu_extra or {}).get(name, []),
            f"-cuid={_file_sha(src)[:16]}", f"-ffile-prefix-map={ROOT}=.",
            f"-ffile-prefix-map={os.path.dirname(os.path.abspath(obj))}=.",
            "-I", os.path.dirname(HEADER), "-I", CSRC, "-c", src, "-o", obj]


def build_library(force: bool = False, extra_flags: list[str] | None = None, out: str = OUT,
                  tu_extra: dict | None = None) -> str:
    """One object per translation unit, compiled in parallel (build/obj/<flags key>), then linked.
    extra_flags: added to every unit (variant builds: -D tunables); tu_extra: {file name: flags}
    for one unit. Objects of builds with different flags never share a directory."""
    if force or needs_build(out, extra_flags, tu_extra):
        from concurrent.futures import ThreadPoolExecutor
        key = _flags_key(out, extra_flags, tu_extra)
        objdir = os.path.join(ROOT, "build", "obj", key)
        os.makedirs(objdir, exist_ok=True)

        def compile_one(src):
            obj = os.path.join(objdir, os.path.basename(src) + ".o")
            subprocess.run(unit_command(src, obj, extra_flags, tu_extra), check=True)
            return obj

        with ThreadPoolExecutor(max_workers=len(SOURCES)) as pool:
            objs = list(pool.map(compile_one, SOURCES))
        subprocess.run([hipcc(), *_arch_flags(), "-shared", "-fPIC", *objs, "-o", out + ".tmp"], check=True)
        os.replace(out + ".tmp", out)
        with open(_stamp_path(out), "w") as f:
            f.write(key + "\n")
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
               f"-ffile-prefix-map={ROOT}=.", COMM_SOURCE, "-o", COMM_OUT + ".tmp", "-L", PKG_DIR, "-ledt_sync",
               "-L", os.path.join(rocm, "lib"), "-lrccl", "-Wl,-rpath,$ORIGIN", "-Wl,-rpath," + os.path.join(rocm, "lib")]
        subprocess.run(cmd, check=True)
        os.replace(COMM_OUT + ".tmp", COMM_OUT)
    return COMM_OUT


if __name__ == "__main__":
    print(build_library(force=True))
    print(build_comm_library(force=True))
