"""bench.py's output contract, checked on the device: ONE JSON line on stdout with the fields the
driver parses (metric / value / unit / n_gpus / steps / warmup / ms_per_step / higher_is_better /
scaling / vs_baseline / dtype / data / config), plus the `roofline` object (bound, achieved, peak,
unit, frac = achieved / peak, traffic) and the `cpu_baseline` object (value, unit, cores, kind,
sample) — for the single-GPU line and for the multi-GPU code path at world 1 (`--sharded`, which
adds roofline.xgmi). Small layout and short budgets: the contract, not the numbers. The printed
line is capped at bench.LINE_CAP characters (the driver keeps only the tail of stdout); the full
record is the sidecar the line names as `detail`, and the sub-object checks read it from there."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
TOP = {"metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
       "vs_baseline", "dtype", "data", "config", "roofline", "cpu_baseline"}


def _run(*extra, full=False):
    import tempfile

    import torch
    if not torch.cuda.is_available():
        pytest.skip("needs a HIP device")
    detail = os.path.join(tempfile.mkdtemp(prefix="edt_bench_"), "detail.json")
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR",
                                                           "MASTER_PORT")}
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--layout", "gpt2_small", "--steps", "3", "--warmup", "1",
           "--cpu-baseline-seconds", "0.4", "--cpu-sample-elems", str(1 << 18), "--ops-cpu-seconds", "0.2",
           "--detail-out", detail, *extra]
    p = subprocess.run(cmd, capture_output=True, text=True, env=env, timeout=110)
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [l for l in p.stdout.splitlines() if l.strip()]
    assert len(lines) == 1, p.stdout              # stdout carries exactly the one JSON line
    assert len(lines[0]) <= 8000, len(lines[0])   # the whole line fits the driver's stdout tail
    line = json.loads(lines[0])
    assert "dropped" not in line, line["dropped"]
    if not full:
        return line
    with open(detail) as f:
        return line, json.load(f)


def _check_common(d, n_gpus):
    assert TOP <= set(d), TOP - set(d)
    assert d["metric"] == "GB/s of param bytes reduced per outer step (device-resident), 1/2/4/8 GPUs"
    assert d["unit"] == "GB/s" and d["n_gpus"] == n_gpus and d["steps"] == 3 and d["warmup"] == 1
    assert d["higher_is_better"] is True and d["scaling"] in ("strong", "weak") and d["vs_baseline"] is None
    assert d["value"] > 0 and d["ms_per_step"] > 0 and d["dtype"] in ("f32", "bf16")
    assert "synthetic" in d["data"] and "workload" in d["config"]
    P = d["config"]["params"]
    # value = K x P x bytes per worker element over the step time
    bw = 4 if d["config"]["worker_dtype"] == "f32" else 2
    assert d["value"] == pytest.approx(d["config"]["population"] * P * bw / (d["ms_per_step"] / 1e3) / 1e9, rel=2e-3)
    r = d["roofline"]
    assert {"bound", "achieved", "peak", "unit", "frac", "traffic"} <= set(r)
    assert r["bound"] == "hbm" and r["unit"] == "GB/s" and r["peak"] == 8000.0
    assert r["frac"] == pytest.approx(r["achieved"] / r["peak"], abs=1e-3) and 0 < r["frac"] < 1
    c = d["cpu_baseline"]
    assert {"value", "unit", "cores", "kind", "sample"} <= set(c) and c["kind"] in ("port", "reference")
    assert c["value"] > 0 and c["cores"] >= 1 and c["sample"]


def test_single_gpu_line():
    d = _run("--place-candidates", "2", "--ops", "none", "--bcast-compare", "0")
    _check_common(d, 1)
    assert d["config"]["parallelism"] == "single GPU"
    assert d["roofline"]["kernel_ms"] <= d["ms_per_step"] * 1.05
    # in-run evidence: the process's own tracer saw the library's fused step kernel
    kt = d["kernel_trace"]
    assert kt["steps"] == 2, kt
    top = kt["kernels"][0]
    assert "outer_kernel<" in top["name"] and top["launches"] == 2, kt
    assert top["mean_ms"] > 0


def test_multi_gpu_path_line_at_world_1():
    d = _run("--gpus", "1", "--sharded", "--compare-schedules", "0", "--config-companions", "0")
    _check_common(d, 1)
    assert "RCCL" in d["config"]["parallelism"]
    x = d["roofline"]["xgmi"]
    assert x["bound"] == "xgmi" and "wire_bytes_per_rank" in x
    assert "weak_scaling" in d and "extras_deadline" not in d
    kt = d["kernel_trace"]
    assert "error" not in kt and any("outer_kernel" in k["name"] for k in kt["kernels"]), kt


def test_single_gpu_line_population_extra():
    """The N = 1 line's BASELINE configs[4] sub-object (population_slerp_7b: 8 members and 8
    children resident, both SLERP forms), here on the 125M layout: fields, roofline arithmetic,
    every lineage tensor in the lerp branch."""
    line, d = _run("--place-candidates", "1", "--ops", "population_7b", "--population-layout", "gpt2_small",
                   "--bcast-compare", "0", full=True)
    _check_common(d, 1)
    _check_common(line, 1)
    p = d["population_slerp_7b"]
    lp = line["population_slerp_7b"]
    assert lp["speculative"]["ms_per_generation"] == p["speculative"]["ms_per_generation"]
    assert lp["gen_ms"]["two_pass"] == [g["two_pass"]["ms"] for g in p["generations"]]
    assert "error" not in p and "skipped" not in p, p
    assert "roulette_wheel_selection" in p["pairs_source"] and p["timed_reps"] >= 10
    gens = p["generations"] + [p["ring"]]
    assert len(p["generations"]) >= 3
    for g in gens:
        assert len(g["pairs"]) == 8 and g["lerp_branch_fraction"] == 1.0
        assert g["distinct_parents"] == len({x for q in g["pairs"] for x in q})
        assert g["layout"]["children"] == 8
        for form in ("speculative", "two_pass"):
            assert g[form]["ms"] > 0 and g[form]["floor_bytes"] > 0
    for form in ("speculative", "two_pass"):
        f = p[form]
        fb = sum(g[form]["floor_bytes"] for g in p["generations"])
        ms = sum(g[form]["ms"] for g in p["generations"])
        assert f["ms_per_generation"] == pytest.approx(ms / len(p["generations"]), rel=1e-3)
        r = f["roofline"]
        assert r["achieved"] == pytest.approx(fb / (ms / 1e3) / 1e9, rel=1e-2)
        assert r["frac"] == pytest.approx(r["achieved"] / r["peak"], abs=1e-3)


def test_single_gpu_line_lm_population_extra():
    """The N = 1 line's EDT-LM generation (lm_population: 8 members of the 1.3B layout resident,
    rank-selected pairs, one edt_pair_merge_population launch per generation): fields and the
    roofline arithmetic over the drawn generations' floor bytes."""
    line, d = _run("--place-candidates", "1", "--ops", "lm_population", "--bcast-compare", "0",
                   "--population-generations", "2", full=True)
    _check_common(d, 1)
    p = d["lm_population"]
    assert line["lm_population"]["gen_ms"] == [g["ms"] for g in p["generations"]]
    assert "error" not in p, p
    assert "rank_based_selection" in p["pairs_source"] and len(p["generations"]) == 2 and p["timed_reps"] >= 10
    fb = sum(g["floor_bytes"] for g in p["generations"])
    ms = sum(g["ms"] for g in p["generations"])
    for g in p["generations"]:
        assert len(g["pairs"]) == 8 and all(a != b for a, b in g["pairs"])
        assert g["distinct_parents"] == len({x for q in g["pairs"] for x in q})
    assert p["roofline"]["achieved"] == pytest.approx(fb / (ms / 1e3) / 1e9, rel=1e-2)
