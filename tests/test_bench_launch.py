"""bench.py's own rank launcher (no torchrun): `--gpus N` without WORLD_SIZE starts N child
processes with the rank environment and stops there under --dry-run-launch (before any device
initialisation), so this runs on a CPU-only host."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.parametrize("n", [2, 4])
def test_bench_spawns_ranks_without_torchrun(n):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR",
                                                           "MASTER_PORT")}
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(n), "--dry-run-launch"],
                       capture_output=True, text=True, env=env, timeout=300)
    assert p.returncode == 0, p.stderr
    lines = [json.loads(l) for l in p.stdout.splitlines() if l.startswith("{")]
    assert sorted(int(l["RANK"]) for l in lines) == list(range(n))
    for l in lines:
        assert l["LOCAL_RANK"] == l["RANK"] and l["WORLD_SIZE"] == str(n)
        assert l["MASTER_ADDR"] == "127.0.0.1"
    assert len({l["MASTER_PORT"] for l in lines}) == 1


def test_bench_launcher_propagates_a_rank_failure():
    """A rank that fails ends the run with its non-zero status: on a host without a GPU every
    rank fails at device selection, after the launcher has started them."""
    import torch
    if torch.cuda.device_count() > 0:
        pytest.skip("needs a host without a GPU (the ranks must fail)")
    env = {k: v for k, v in os.environ.items() if k != "WORLD_SIZE"}
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "1"],
                       capture_output=True, text=True, env=env, timeout=300)
    assert p.returncode != 0
    assert p.stderr.count("Traceback") >= 1


def _alive(pid):
    try:
        os.kill(pid, 0)
    except ProcessLookupError:
        return False
    with open(f"/proc/{pid}/stat") as f:          # a zombie is gone for our purpose
        return f.read().split(")")[-1].split()[0] != "Z"


@pytest.mark.parametrize("how", ["term", "kill"])
def test_bench_launcher_takes_its_ranks_down(how):
    """A launcher stopped by SIGTERM forwards it and waits for its ranks; one killed outright
    (SIGKILL: no handler runs) still takes them with it (PR_SET_PDEATHSIG). Either way no rank is
    left running, as a timed-out driver run must not leave ranks holding GPUs."""
    import signal
    import time
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR",
                                                           "MASTER_PORT")}
    p = subprocess.Popen([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--dry-run-launch",
                          "--dry-run-sleep", "120"], stdout=subprocess.PIPE, text=True, env=env)
    pids = [json.loads(p.stdout.readline())["PID"] for _ in range(2)]
    assert all(_alive(q) for q in pids)
    p.send_signal(signal.SIGTERM if how == "term" else signal.SIGKILL)
    p.wait(timeout=60)
    deadline = time.time() + 30
    while time.time() < deadline and any(_alive(q) for q in pids):
        time.sleep(0.1)
    assert not any(_alive(q) for q in pids)
    if how == "term":
        assert p.returncode == 128 + signal.SIGTERM
