"""The whole N > 1 bench line rehearsed on the CPU, so the driver's first multi-GPU run cannot die in
untried host code (EDT_LM/diloco.py:231-235,302-308 is the exchange it replaces).

bench.run_sharded — the function `python bench.py --gpus N` runs on every rank — driven here over
gloo at world 2 and 4 by real rank processes (the same environment the launcher gives them), with
the CPU stand-in kernels injected by this test (tests/oracle_kernels.py; the product ops stay the
default in bench.py) and tiny layouts registered for the run. Every extra runs: the weak
companion, the other schedules, BASELINE configs[2]/[3] (tiny layouts here) and configs[4]'s
population crossover; and the extras deadline fires on a rank that hangs, which must still print
the line with the value and exit non-zero."""
import json
import os
import socket
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

LAYOUTS = {"rehearsal_main": [(64, 33), (257,), (31, 17), (1000,)],
           "rehearsal_parity": [(61, 37), (129,), (5,), (3000,)],
           "rehearsal_c2": [(40, 24), (24,), (333,)],
           "rehearsal_c3": [(128, 9), (77,)],
           "rehearsal_pop": [(300,), (17, 19), (1024,)]}
ARGS = ["--layout", "rehearsal_main", "--population", "4", "--steps", "2", "--warmup", "1",
        "--cpu-baseline-seconds", "0.2", "--cpu-sample-elems", "4096", "--bucket-elems", "2048",
        "--config-layouts", "configs2_125m_fp32=rehearsal_c2:f32,configs3_1p3b_bf16=rehearsal_c3:bf16",
        "--population-layout", "rehearsal_pop", "--population-groups", "2",
        "--parity-layout", "rehearsal_parity", "--parity-bucket-elems", "1024"]


def _rank_main():
    """One rank (launched by _launch with the torchrun-style environment)."""
    import time

    import torch
    import torch.distributed as dist
    sys.path.insert(0, ROOT)
    import bench
    from evolutionarydistributedtraining_amd.collectives import TorchCollectives
    from evolutionarydistributedtraining_amd.layouts import LAYOUTS as REG
    from evolutionarydistributedtraining_amd.params import ParamLayout
    from oracle import oracle
    from tests.oracle_kernels import ChunkGramKernels, OracleKernels
    for name, shapes in LAYOUTS.items():
        REG[name] = lambda shapes=shapes: ParamLayout(shapes)
    hang_rank = int(os.environ.get("REHEARSAL_HANG_RANK", "-1"))

    class Kernels(ChunkGramKernels):
        def slerp_arena(self, plan, v0, v1, out, t, thr=0.9995, eps=1e-8, **kw):
            OracleKernels.slerp_arena(self, getattr(plan, "seg_offsets", plan), v0, v1, out, t, thr, eps)

        def slerp_needed_sums(self, members, layout, chunks, nchunks, table, row0, scratch=None):
            if dist.get_rank() == hang_rank:
                time.sleep(120)                  # a peer that never answers: the deadline must fire
            return super().slerp_needed_sums(members, layout, chunks, nchunks, table, row0, scratch)

    class Corrupting(TorchCollectives):
        """Every received buffer's first element nudged after the collective lands: what a
        collective that moved wrong bytes looks like to the schedule (REHEARSAL_CORRUPT=1)."""

        def _after(self, work, out, async_op):
            def nudge():
                if out.numel():
                    out.view(-1)[0] += 1
            if not async_op:
                nudge()
                return work

            class W:
                def wait(self_inner):
                    work.wait()
                    nudge()
            return W()

        def all_gather(self, out, inp, async_op=False):
            return self._after(super().all_gather(out, inp, async_op), out, async_op)

        def all_to_all(self, out, inp, async_op=False):
            return self._after(super().all_to_all(out, inp, async_op), out, async_op)

        def reduce_scatter(self, out, inp, async_op=False):
            return self._after(super().reduce_scatter(out, inp, async_op), out, async_op)

    torch.set_num_threads(2)
    dist.init_process_group("gloo", rank=int(os.environ["RANK"]), world_size=int(os.environ["WORLD_SIZE"]))
    args = bench.parse(json.loads(os.environ["REHEARSAL_ARGS"]))
    comm = Corrupting() if os.environ.get("REHEARSAL_CORRUPT") == "1" else TorchCollectives()
    bench.run_sharded(args, comm, bench.Runtime("cpu"), sys.stdout, kernels=Kernels(oracle))
    dist.destroy_process_group()


def _launch(world, extra=(), hang_rank=-1, timeout=240, corrupt=False):
    import tempfile
    detail = os.path.join(tempfile.mkdtemp(prefix="edt_rehearsal_"), "detail.json")
    extra = ["--detail-out", detail] + list(extra)
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    procs = []
    for r in range(world):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(world), MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port), REHEARSAL_ARGS=json.dumps(ARGS + ["--gpus", str(world)] + list(extra)),
                   REHEARSAL_HANG_RANK=str(hang_rank), OMP_NUM_THREADS="2",
                   REHEARSAL_CORRUPT="1" if corrupt else "0")
        procs.append(subprocess.Popen([sys.executable, "-c", "from tests.test_bench_rehearsal import _rank_main; "
                                       "_rank_main()"], cwd=ROOT, env=env, stdout=subprocess.PIPE,
                                      stderr=subprocess.PIPE, text=True))
    outs = []
    try:
        for p in procs:
            o, e = p.communicate(timeout=timeout)
            outs.append((p.returncode, o, e))
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
    lines = [l for l in outs[0][1].splitlines() if l.startswith("{")]
    for l in lines:                  # the whole line fits the driver's stdout tail
        assert len(l) <= 8000, len(l)
    if lines and os.path.exists(detail):     # the printed line is the compact projection:
        with open(detail) as f:              # tests read the full record from the sidecar
            full = json.load(f)
        lines = [json.dumps(dict(full, line=json.loads(lines[0])))]
    return outs, lines


def bench_link_gbps():
    sys.path.insert(0, ROOT)
    import bench
    return bench.XGMI_LINK_GBPS


@pytest.mark.slow
@pytest.mark.parametrize("world", [2, 4, 8])
def test_bench_line_at_world(world):
    """world 8: the driver's node (population 8, one worker per rank; `auto` takes exact there)."""
    outs, lines = _launch(world, extra=["--population", "8"] if world == 8 else ())
    assert all(rc == 0 for rc, _, _ in outs), [(rc, e[-2000:]) for rc, _, e in outs]
    assert len(lines) == 1, outs[0][1][-2000:]
    for rc, o, _ in outs[1:]:
        assert not [l for l in o.splitlines() if l.startswith("{")]        # only rank 0 prints
    d = json.loads(lines[0])
    assert d["n_gpus"] == world and d["value"] >= 0 and d["ms_per_step"] > 0     # tiny layout: ~0 GB/s
    assert d["roofline"]["xgmi"]["wire_bytes_per_rank"] > 0
    line = d["line"]
    assert "dropped" not in line and line["detail"].endswith("detail.json")
    # the first hardware line states its own exchange floor (wire bytes / (N-1) links)
    x = line["roofline"]["xgmi"]
    assert x["floor_ms"] == pytest.approx(x["wire_bytes_per_rank"] / (bench_link_gbps() * (world - 1) * 1e9) * 1e3,
                                          abs=1e-4)
    assert all("xgmi_floor_ms" in v for v in line["other_schedules"].values())
    assert line["population_slerp_7b"]["sharded"]["parity"]["bit_exact"] is True
    assert d["roofline"]["kernel_ms"] > 0 and d["roofline"]["algo_bytes_per_launch"] > 0
    assert d["cpu_baseline"]["value"] > 0 and "c_port" in d["cpu_baseline"]
    for key in ("weak_scaling", "other_schedules", "baseline_configs", "population_slerp_7b"):
        assert key in d, key
    assert "error" not in d["weak_scaling"], d["weak_scaling"]
    assert len(d["other_schedules"]) == 3 and all("error" not in v for v in d["other_schedules"].values()), \
        d["other_schedules"]
    assert set(d["baseline_configs"]) == {"configs2_125m_fp32", "configs3_1p3b_bf16"}
    assert all("error" not in v for v in d["baseline_configs"].values()), d["baseline_configs"]
    pop = d["population_slerp_7b"]
    assert "error" not in pop and {"sharded", "sharded_pipelined", "per_child"} <= set(pop), pop
    assert pop["sharded"]["wire_bytes_per_rank"] > 0
    assert "roulette_wheel_selection" in pop["pairs_source"] and len(pop["pairs"]) == world
    tab = pop["sums_table"]                    # r5: only the needed sums are formed and gathered
    assert 0 < tab["sums_per_chunk"] <= tab["triangle_sums_per_chunk"], tab
    assert "extras_deadline" not in d
    par = d["parity"]                          # the exchange moved the right bytes
    assert "error" not in par, par
    assert par["bit_exact"] and par["max_ulp"] == 0 and par["replicas_identical"], par
    assert par["replicas_equal_reference"] and par["buckets"] > 1 and par["schedule"] == d["config"]["parallelism"].split()[1]
    assert pop["sharded"]["parity"]["bit_exact"], pop["sharded"]
    assert pop["sharded_pipelined"]["parity"]["bit_exact"], pop["sharded_pipelined"]
    if world == 8:
        assert d["config"]["parallelism"].startswith("dp8 exact/"), d["config"]


@pytest.mark.slow
@pytest.mark.parametrize("corrupt", [False, True])
@pytest.mark.parametrize("mode,world", [("exact", 2), ("reduce_ordered", 2), ("reduce_ordered", 3)])
def test_bench_parity_per_schedule(mode, world, corrupt):
    """The parity record of each bit-exact schedule: clean collectives give the single-GPU kernels'
    bits; a collective that delivers one wrong element per buffer leaves the value reported but
    flips the record (so the driver's first 8-GPU line is evidence of correctness, not only of
    speed)."""
    outs, lines = _launch(world, extra=["--mode", mode, "--broadcast", "theta", "--compare-schedules", "0",
                                        "--config-companions", "0", "--weak-companion", "0", "--ops", "",
                                        "--population", "6"], corrupt=corrupt)
    assert all(rc == 0 for rc, _, _ in outs), [(rc, e[-2000:]) for rc, _, e in outs]
    d = json.loads(lines[0])
    par = d["parity"]
    assert par["schedule"] == f"{mode}/theta" and par["workers"] == 6, par
    if corrupt:
        assert not par["bit_exact"] and par["max_ulp"] > 0 and not par["replicas_equal_reference"], par
    else:
        assert par["bit_exact"] and par["max_ulp"] == 0 and par["replicas_equal_reference"], par


@pytest.mark.slow
def test_bench_line_deadline_fires_on_a_hung_rank():
    """Rank 0 hangs inside the population crossover (the last extra): the deadline prints the line
    with the value and every finished extra, names the unfinished one, and every rank exits 3."""
    outs, lines = _launch(2, extra=["--extras-deadline", "20"], hang_rank=0)
    assert [rc for rc, _, _ in outs] == [3, 3], [(rc, e[-1500:]) for rc, _, e in outs]
    assert len(lines) == 1
    d = json.loads(lines[0])
    assert d["ms_per_step"] > 0 and d["cpu_baseline"]["value"] > 0
    assert {"weak_scaling", "other_schedules", "baseline_configs"} <= set(d)
    assert d["extras_deadline"]["unfinished_or_skipped"] == ["population_slerp_7b"]
