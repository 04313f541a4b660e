"""The drop-in files under integration/ (copies of the reference's three crossover.py entry points)
work where the reference keeps them: copied into a directory of their own, run as the workers run
them (`python crossover.py --model1_path …`, EDT_LM/edt.py / EDT_EVOMERGE/edt.py:262-280) or
imported as the RL master imports them (`from crossover import crossover`, EDT_RL/edt.py:6),
finding this package through EDT_SYNC_ROOT — and failing with a clear message when they cannot.
No GPU: `--help` and the import stop before any device work."""
import os
import shutil
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _env(with_root=True):
    env = {k: v for k, v in os.environ.items() if k not in ("PYTHONPATH", "EDT_SYNC_ROOT")}
    if with_root:
        env["EDT_SYNC_ROOT"] = ROOT
    return env


def _copy(tmp_path, rel):
    d = tmp_path / "train"
    d.mkdir()
    shutil.copy(os.path.join(ROOT, "integration", rel), d / "crossover.py")
    return d


@pytest.mark.parametrize("rel", ["EDT_LM/train/crossover.py", "EDT_EVOMERGE/train/crossover.py"])
def test_worker_cli_shims(tmp_path, rel):
    d = _copy(tmp_path, rel)
    p = subprocess.run([sys.executable, "crossover.py", "--help"], cwd=d, env=_env(), capture_output=True, text=True,
                       timeout=300)
    assert p.returncode == 0, p.stderr
    for flag in ("--model1_path", "--model2_path", "--output_path"):
        assert flag in p.stdout


def test_rl_master_import_shim(tmp_path):
    d = _copy(tmp_path, "EDT_RL/crossover.py")
    code = ("from crossover import crossover, slerp, lerp, normalize, interpolate_t, run_slerp_merge_from_config; "
            "print(interpolate_t(1, 4, [0, 0.5, 0.3, 0.7, 1]))")
    p = subprocess.run([sys.executable, "-c", code], cwd=d, env=_env(), capture_output=True, text=True, timeout=300)
    assert p.returncode == 0, p.stderr
    assert abs(float(p.stdout.strip()) - 0.43333) < 1e-4


def test_shim_without_the_package_says_how_to_find_it(tmp_path):
    d = _copy(tmp_path, "EDT_RL/crossover.py")
    p = subprocess.run([sys.executable, "-c", "import crossover"], cwd=d, env=_env(with_root=False),
                       capture_output=True, text=True, timeout=300)
    assert p.returncode != 0 and "EDT_SYNC_ROOT" in p.stderr
