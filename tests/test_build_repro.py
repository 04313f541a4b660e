"""The library stamp is source-determined: a translation unit built at two
different checkout paths gives identical objects, so `libedt_sync.so`'s sha256 — the stamp that
gates `roofline.traffic` in bench.py (`_pmc_traffic`) — names the source, not the build path.
Compiles one small unit (edt_merge.hip) at two roots with build.unit_command; no GPU needed."""
import hashlib
import os
import shutil
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HIPCC = "/opt/rocm/bin/hipcc"


def _sha(path):
    with open(path, "rb") as f:
        return hashlib.sha256(f.read()).hexdigest()


@pytest.mark.skipif(not os.path.exists(HIPCC), reason="hipcc not installed")
def test_object_identical_at_two_roots(tmp_path):
    shas = []
    for root in (tmp_path / "a", tmp_path / "b" / "deeper" / "path"):
        pkg = root / "evolutionarydistributedtraining_amd"
        shutil.copytree(os.path.join(ROOT, "include"), root / "include")
        shutil.copytree(os.path.join(ROOT, "evolutionarydistributedtraining_amd", "csrc"), pkg / "csrc")
        shutil.copy(os.path.join(ROOT, "evolutionarydistributedtraining_amd", "build.py"), pkg / "build.py")
        (pkg / "__init__.py").write_text("")
        code = ("import sys, subprocess; sys.path.insert(0, '.');"
                "from evolutionarydistributedtraining_amd import build as b;"
                "src = b.os.path.join(b.CSRC, 'edt_merge.hip');"
                "subprocess.run(b.unit_command(src, 'obj/edt_merge.o'), check=True)")
        (root / "obj").mkdir()
        subprocess.run([sys.executable, "-c", code], cwd=root, check=True, capture_output=True)
        shas.append(_sha(root / "obj" / "edt_merge.o"))
    assert shas[0] == shas[1]


def test_unit_command_fixes_cuid_and_paths():
    from evolutionarydistributedtraining_amd import build as b
    src = os.path.join(b.CSRC, "edt_outer.hip")
    cmd = b.unit_command(src, "/tmp/x/edt_outer.o")
    assert f"-cuid={_sha(src)[:16]}" in cmd
    assert f"-ffile-prefix-map={b.ROOT}=." in cmd
    # the link step takes its arch from the same flag list as the units
    assert b._arch_flags() == [f for f in b.HIPCC_FLAGS if f.startswith("--offload-arch=")]


def test_flag_change_forces_rebuild(tmp_path):
    from evolutionarydistributedtraining_amd import build as b
    out = str(tmp_path / "libx.so")
    with open(out, "wb") as f:
        f.write(b"x")
    with open(out + ".flags", "w") as f:
        f.write(b._flags_key(out, None, None) + "\n")
    os.utime(out, (4e9, 4e9))                    # newer than every source
    assert not b.needs_build(out)
    assert b.needs_build(out, extra_flags=["-DEDT_VARIANT=1"])
    assert b._flags_key(out, ["-DA"], None) != b._flags_key(str(tmp_path / "liby.so"), ["-DA"], None)
