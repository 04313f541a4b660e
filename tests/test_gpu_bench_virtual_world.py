"""The whole N > 1 bench line with the product HIP kernels: bench.run_sharded — what every rank of
`python bench.py --gpus N` runs — on N virtual ranks (collectives.VirtualWorld: threads of one
process sharing this box's one GPU) instead of N processes over RCCL. tests/test_bench_rehearsal.py
drives the same function over gloo with CPU stand-in kernels; here the schedules' kernels are the
library's (edt_outer_step partials, sgd_apply, the population's needed-sums passes), so the
driver's first 8-GPU line meets no untried pairing of host code and device kernels. Only the
transport differs (VirtualCollectives: device copies / adds in rank order)."""
import io
import json
import os
import sys

import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0")

LAYOUTS = {"vw_main": [(640, 330), (2570,), (310, 170), (10000,)],
           "vw_parity": [(61, 37), (129,), (5,), (3000,)],
           "vw_c2": [(400, 240), (240,), (3330,)],
           "vw_c3": [(1280, 90), (770,)],
           "vw_pop": [(3000,), (170, 190), (10240,)]}
ARGS = ["--layout", "vw_main", "--steps", "3", "--warmup", "1", "--kernel-trace", "0",
        "--cpu-baseline-seconds", "0.2", "--cpu-sample-elems", "4096", "--bucket-elems", "32768",
        "--config-layouts", "configs2_125m_fp32=vw_c2:f32,configs3_1p3b_bf16=vw_c3:bf16",
        "--population-layout", "vw_pop", "--population-groups", "2",
        "--parity-layout", "vw_parity", "--parity-bucket-elems", "1024"]


@pytest.fixture(scope="module", autouse=True)
def layouts():
    from evolutionarydistributedtraining_amd.layouts import LAYOUTS as REG
    from evolutionarydistributedtraining_amd.params import ParamLayout
    for name, shapes in LAYOUTS.items():
        REG[name] = lambda shapes=shapes: ParamLayout(shapes)
    yield
    for name in LAYOUTS:
        REG.pop(name, None)


class _Exit(Exception):
    pass


def _run(world, tmp_path, extra=()):
    import bench
    from evolutionarydistributedtraining_amd.collectives import VirtualWorld
    detail = str(tmp_path / "detail.json")
    args = bench.parse(ARGS + ["--gpus", str(world), "--detail-out", detail] + list(extra))
    outs = [io.StringIO() for _ in range(world)]

    def exit_fn(code):                      # the deadline must not end the test process
        raise _Exit(code)

    def body(comm):
        return bench.run_sharded(args, comm, bench.Runtime(DEV), outs[comm.rank], exit_fn=exit_fn)

    res = VirtualWorld(world, timeout=150).run(body)
    torch.cuda.synchronize()
    lines = [l for l in outs[0].getvalue().splitlines() if l.startswith("{")]
    assert len(lines) == 1 and all(not o.getvalue().strip() for o in outs[1:])
    assert len(lines[0]) <= 8000
    with open(detail) as f:                 # the printed line is the projection of this record
        assert json.load(f)["value"] == json.loads(lines[0])["value"]
    return res[0], json.loads(lines[0])


@pytest.mark.parametrize("world", [2, 4])
def test_bench_line_on_virtual_ranks_with_the_hip_kernels(world, tmp_path):
    full, line = _run(world, tmp_path, ["--population", "8" if world == 4 else "4"])
    assert line["n_gpus"] == world and full["ms_per_step"] > 0
    roof = full["roofline"]
    assert roof["kernel_ms"] > 0 and roof["algo_bytes_per_launch"] > 0
    assert roof["xgmi"]["wire_bytes_per_rank"] > 0 and roof["xgmi"]["floor_ms"] is not None
    par = full["parity"]                    # the exchange moved the right bytes through real kernels
    assert "error" not in par, par
    assert par["bit_exact"] and par["max_ulp"] == 0 and par["replicas_identical"], par
    assert par["replicas_equal_reference"] and par["buckets"] > 1, par
    assert "error" not in full["weak_scaling"], full["weak_scaling"]
    assert len(full["other_schedules"]) == 3, full["other_schedules"]
    assert all("error" not in v for v in full["other_schedules"].values()), full["other_schedules"]
    assert all("error" not in v for v in full["baseline_configs"].values()), full["baseline_configs"]
    pop = full["population_slerp_7b"]
    assert "error" not in pop, pop
    assert pop["sharded"]["parity"]["bit_exact"], pop["sharded"]
    assert pop["sharded_pipelined"]["parity"]["bit_exact"], pop["sharded_pipelined"]
    assert "extras_deadline" not in full


@pytest.mark.parametrize("mode", ["exact", "reduce_ordered", "reduce"])
def test_bench_schedule_parity_on_virtual_ranks(mode, tmp_path):
    """Each schedule as the timed one: exact and reduce_ordered bit-exact against the single-GPU
    fused step; reduce (the transport's summation order: ulps, not bits) with every replica
    identical."""
    full, _ = _run(2, tmp_path, ["--mode", mode, "--broadcast", "theta", "--compare-schedules", "0",
                                 "--config-companions", "0", "--weak-companion", "0", "--ops", "", "--population", "6"])
    par = full["parity"]
    assert "error" not in par and par["schedule"] == f"{mode}/theta", par
    if mode == "reduce":
        assert par["replicas_identical"], par
    else:
        assert par["bit_exact"] and par["max_ulp"] == 0 and par["replicas_equal_reference"], par
