"""Benchmark: DiLoCo outer step (fused delta + population mean + Nesterov SGD) on MI355X.

Metric (BASELINE.json): "GB/s of param bytes reduced per outer step (device-resident)".
  value = (total workers K) x P x (bytes per worker element) / (wall time of one step),
  aggregated over all ranks.

Default workload (N=1): the 1.3B-parameter GPT layout (P = 1,315,723,264, 292 tensors), a
population of 8 workers resident on the GPU, everything fp32 — the dtype the reference computes
the outer step in as written (transformers 4.x `from_pretrained` loads fp32) —
and diloco.py's outer optimiser (lr 0.7, momentum 0.9, Nesterov) in steady state (carried
buffer). `--theta-dtype bf16 --worker-dtype bf16` is the all-bf16 form (transformers 5.x, BASELINE
cfg4's "bf16 params"); `--worker-dtype bf16` alone keeps an fp32 master with bf16 replicas.
N>1 (BASELINE configs "8 workers over 8 GPUs"): the population stays K = 8 and
is spread 8/N workers per GPU (strong scaling); the cross-replica step runs over RCCL (xGMI):
reduce-scatter of fp32 partial sums + sharded SGD + all-gather of theta, or all-to-all of the raw
worker shards + the fused kernel per shard (bit-exact) + all-gather of the new theta rounded to
bf16 straight into the worker arenas (the fp32 master stays sharded), whichever puts fewer bytes
on the wire (distributed.py).
`--workers-per-gpu W` instead fixes W workers per GPU (weak scaling, population W*N).

    python bench.py [--gpus N --steps K --warmup W]
    torchrun --nproc-per-node N --master-addr 127.0.0.1 bench.py --gpus N ...

Prints ONE JSON line on rank 0. Also reports the fused kernel's own duration (HIP events on the
stream it is launched on), the HBM roofline fraction, and the CPU oracle timed on this host.
At N=1, after the warm-up steps and before the timed ones, the momentum buffer's HBM placement is
chosen by measurement (OuterSync.place_momentum, placement.py: the step's two read-modify-write
streams run up to 11 % faster or slower depending on their relative physical placement); the
candidates' probe times are in roofline.momentum_placement, and --place-candidates 1 disables it.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBPS = 8000.0        # MI355X HBM3E spec peak (MI355X_MICROARCH.md)
XGMI_LINK_GBPS = 153.6 / 2    # per xGMI link and direction (153.6 GB/s both ways); 7 links per GPU, one to each peer
DT = {"f32": torch.float32, "bf16": torch.bfloat16}


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=20)
    p.add_argument("--warmup", type=int, default=5)
    p.add_argument("--layout", default="gpt_1p3b")
    p.add_argument("--population", type=int, default=8, help="total workers K (strong scaling)")
    p.add_argument("--workers-per-gpu", type=int, default=None, help="fixed per GPU (weak scaling)")
    p.add_argument("--theta-dtype", default="f32", choices=DT)
    p.add_argument("--worker-dtype", default="f32", choices=DT)
    p.add_argument("--lr", type=float, default=0.7)
    p.add_argument("--momentum", type=float, default=0.9)
    p.add_argument("--nesterov", type=int, default=1)
    p.add_argument("--mode", default="auto", choices=["reduce", "exact", "auto"])
    p.add_argument("--broadcast", default="auto", choices=["theta", "workers", "auto"],
                   help="N>1: all-gather the fp32 theta replica, or the new theta rounded into the "
                        "worker arenas (fp32 master kept sharded)")
    p.add_argument("--bucket-elems", type=int, default=1 << 26)
    p.add_argument("--cpu-baseline-seconds", type=float, default=10.0)
    p.add_argument("--cpu-sample-elems", type=int, default=1 << 24)
    p.add_argument("--sharded", action="store_true",
                   help="run the multi-GPU (RCCL) schedule even at world size 1 (launch with torchrun)")
    p.add_argument("--weak-companion", type=int, default=1,
                   help="N>1: after the timed strong-scaling steps, also time W = population workers per GPU "
                        "(weak scaling) and report it beside the value as 'weak_scaling'")
    p.add_argument("--place-candidates", type=int, default=8,
                   help="N=1: choose the momentum buffer's HBM placement among this many allocations by "
                        "timing the step's access pattern on each, once before the timed steps (placement.py); "
                        "1 keeps the first allocation")
    p.add_argument("--traffic-json", default=os.path.join(ROOT, "profiles", "pmc_traffic.json"))
    return p.parse_args()


def synth_population(theta: torch.Tensor, workers: list[torch.Tensor], seed: int) -> None:
    """theta ~ N(0, 0.02^2); worker k = theta + N(0, 1e-3^2), on the device."""
    g = torch.Generator(device=theta.device).manual_seed(seed)
    chunk = 1 << 26
    n = theta.numel()
    for a in range(0, n, chunk):
        b = min(n, a + chunk)
        t = torch.randn(b - a, generator=g, device=theta.device) * 0.02
        theta[a:b].copy_(t)
        for w in workers:
            w[a:b].copy_(t + torch.randn(b - a, generator=g, device=theta.device) * 1e-3)


def cpu_baseline(args, theta_dtype, worker_dtype, k):
    """The CPU oracle (the reference's op sequence restated in C, OpenMP) on a bounded sample."""
    from oracle import oracle
    n = args.cpu_sample_elems
    g = torch.Generator().manual_seed(1)
    theta = (torch.randn(n, generator=g) * 0.02).to(theta_dtype)
    workers = [(theta.float() + torch.randn(n, generator=g) * 1e-3).to(worker_dtype) for _ in range(k)]
    mom = torch.zeros(n, dtype=theta_dtype)
    oracle.outer_step(theta, workers, mom, False, args.lr, args.momentum, bool(args.nesterov))
    times = []
    t_end = time.perf_counter() + args.cpu_baseline_seconds
    while time.perf_counter() < t_end or len(times) < 2:
        t0 = time.perf_counter()
        oracle.outer_step(theta, workers, mom, True, args.lr, args.momentum, bool(args.nesterov))
        times.append(time.perf_counter() - t0)
    times.sort()
    t = times[len(times) // 2]
    gbps = k * n * torch.finfo(worker_dtype).bits / 8 / t / 1e9
    out = {"value": round(gbps, 3), "unit": "GB/s", "cores": oracle.max_threads(), "kind": "port",
           "sample": f"{n} elements x {k} workers (fused delta+mean+SGD, oracle/edt_oracle.c, "
                     f"median of {len(times)} reps over {args.cpu_baseline_seconds:.0f}s)"}
    del theta, workers, mom
    out["reference_loop"] = reference_loop_baseline(args, theta_dtype, worker_dtype, k)
    return out


def reference_loop_baseline(args, theta_dtype, worker_dtype, k):
    """The reference's outer step as it runs on its master's CPU (per-tensor torch ops + SGD,
    restated in oracle.torch_loop_outer_step) over the first tensors of the bench layout, up to
    the same element budget: the cost the fused kernel replaces, next to the C port above."""
    from evolutionarydistributedtraining_amd.layouts import LAYOUTS
    from oracle import oracle
    shapes, total = [], 0
    for shp in LAYOUTS[args.layout]().shapes:         # in order, skipping what would overflow
        m = int(torch.Size(shp).numel())
        if total + m <= args.cpu_sample_elems:
            shapes.append(shp)
            total += m
    g = torch.Generator().manual_seed(2)
    base = [(torch.randn(shp, generator=g) * 0.02).to(theta_dtype) for shp in shapes]
    workers = [[(p.float() + torch.randn(p.shape, generator=g) * 1e-3).to(worker_dtype) for p in base]
               for _ in range(k)]
    opt = oracle.torch_loop_outer_step(base, workers, None, args.lr, args.momentum, bool(args.nesterov))
    times = []
    t_end = time.perf_counter() + args.cpu_baseline_seconds / 2
    while time.perf_counter() < t_end or len(times) < 2:
        t0 = time.perf_counter()
        opt = oracle.torch_loop_outer_step(base, workers, opt, args.lr, args.momentum, bool(args.nesterov))
        times.append(time.perf_counter() - t0)
    times.sort()
    t = times[len(times) // 2]
    return {"value": round(k * total * torch.finfo(worker_dtype).bits / 8 / t / 1e9, 3), "unit": "GB/s",
            "threads": torch.get_num_threads(),
            "sample": f"{len(shapes)} tensors of {args.layout} in order ({total} elements) x {k} workers, "
                      f"EDT_LM/diloco.py:238-289's per-tensor torch loop + torch.optim.SGD "
                      f"(oracle.torch_loop_outer_step), median of {len(times)} reps"}


def stream_ceiling_ms(theta, workers, momentum, iters=10):
    """Median HIP-event time of edt_probe_stream over the step's own operands (None if the
    step runs without momentum: the probe always reads and writes a momentum stream)."""
    if momentum is None or len(workers) > 64:    # the probe is one launch (<= 64 workers)
        return None
    from evolutionarydistributedtraining_amd import _lib as L
    lib = L.lib()
    arr = L.ptr_array(workers)
    st = L.stream_ptr(theta.device)
    call = lambda: L.check(lib.edt_probe_stream(L.ptr(theta), L.dtype_code(theta), arr, L.dtype_code(workers[0]),
                                                len(workers), L.ptr(momentum), theta.numel(), st), "edt_probe_stream")
    call()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(iters)]
    for a, b in ev:
        a.record()
        call()
        b.record()
    torch.cuda.synchronize()
    ts = sorted(a.elapsed_time(b) for a, b in ev)
    return ts[len(ts) // 2]


def time_sharded(args, layout, tdt, wdt, k_local, dev, rank, steps, warmup):
    """Build a ShardedOuterSync with k_local workers per rank, warm it up and time `steps` steps
    (barrier + synchronize on both sides, max over ranks). Returns (ms_per_step, mode/broadcast,
    wire bytes per rank); frees the arenas."""
    import torch.distributed as dist
    from evolutionarydistributedtraining_amd.distributed import ShardedOuterSync
    sync = ShardedOuterSync(layout, tdt, wdt, k_local, dev, args.lr, args.momentum, bool(args.nesterov),
                            mode=args.mode, bucket_elems=args.bucket_elems, broadcast=args.broadcast)
    synth_population(sync.theta.flat, [w.flat for w in sync.workers], seed=4321 + 7919 * rank)
    dist.broadcast(sync.theta_buf, 0)
    for _ in range(warmup):
        sync.step()
    torch.cuda.synchronize()
    dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        sync.step()
    torch.cuda.synchronize()
    dist.barrier()
    t = torch.tensor([time.perf_counter() - t0], device=dev, dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    res = (t.item() / steps * 1e3, f"{sync.mode}/{sync.broadcast}", sync.wire_bytes())
    del sync
    torch.cuda.empty_cache()
    return res


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        if not (world == 1 and args.gpus == 1):
            raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}: launch with torchrun")
    torch.cuda.set_device(local)
    sharded = world > 1 or args.sharded    # --sharded: the multi-GPU code path on one rank
    dev = torch.device("cuda", local)
    import torch.distributed as dist
    if sharded:
        dist.init_process_group("nccl", device_id=dev)

    from evolutionarydistributedtraining_amd import ops
    from evolutionarydistributedtraining_amd.layouts import LAYOUTS
    from evolutionarydistributedtraining_amd.diloco import OuterSync
    from evolutionarydistributedtraining_amd.params import ParamArena

    layout = LAYOUTS[args.layout]()
    tdt, wdt = DT[args.theta_dtype], DT[args.worker_dtype]
    if args.workers_per_gpu:
        k_local, scaling = args.workers_per_gpu, "weak"
    else:
        if args.population % world:
            raise SystemExit(f"population {args.population} does not split over {world} GPUs")
        k_local, scaling = args.population // world, "strong"
    k_total = k_local * world
    P = layout.total
    if not sharded:
        theta = ParamArena(layout, tdt, dev)
        workers = [ParamArena(layout, wdt, dev) for _ in range(k_local)]
        synth_population(theta.flat, [w.flat for w in workers], seed=1234)
        sync = OuterSync(theta, workers, args.lr, args.momentum, bool(args.nesterov))
        step = sync.step
        kernel_name = "outer_kernel"
    else:
        from evolutionarydistributedtraining_amd.distributed import ShardedOuterSync
        sync = ShardedOuterSync(layout, tdt, wdt, k_local, dev, args.lr, args.momentum, bool(args.nesterov),
                                mode=args.mode, bucket_elems=args.bucket_elems, broadcast=args.broadcast)
        synth_population(sync.theta.flat, [w.flat for w in sync.workers], seed=1234 + 7919 * rank)
        # replicas of theta must agree: rank 0's values everywhere
        dist.broadcast(sync.theta_buf, 0)
        step = sync.step
        kernel_name = "outer_kernel" if sync.mode == "exact" else "outer_kernel(partial)"

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    placement = None
    if not sharded and args.place_candidates > 1:
        # once per run, outside the timed region: the momentum buffer goes wherever the step's
        # access pattern runs fastest (placement.py); every later step uses that placement
        try:
            placement = sync.place_momentum(args.place_candidates)
        except Exception as e:          # a measurement extra: report it, keep the first allocation
            placement = {"error": f"{type(e).__name__}: {e}"}
        step()
        torch.cuda.synchronize()

    # fused-kernel duration, measured with HIP events on the launch stream (torch's current)
    kern_ms = None
    if not sharded:
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(args.steps)]

    if sharded:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(args.steps):
        if not sharded:
            ev[i][0].record()
        step()
        if not sharded:
            ev[i][1].record()
    torch.cuda.synchronize()
    if sharded:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if sharded:
        t = torch.tensor([elapsed], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = t.item()
    ms_per_step = elapsed / args.steps * 1e3
    if not sharded:
        ks = sorted(a.elapsed_time(b) for a, b in ev)
        kern_ms = sum(ks) / len(ks)

    bytes_reduced = k_total * P * torch.finfo(wdt).bits // 8
    value = bytes_reduced / (ms_per_step / 1e3) / 1e9

    sched = f"{sync.mode}/{sync.broadcast}" if sharded else None
    wire_main = sync.wire_bytes() if sharded else None
    weak = None
    if sharded and scaling == "strong" and args.weak_companion:     # (world 1: --sharded rehearsal)
        # the same schedule with the N = 1 population on EVERY rank (population x N): per-GPU work
        # fixed, so value_N / (N value_1) isolates the cost of the xGMI exchange
        del sync, step
        torch.cuda.empty_cache()
        try:
            w_ms, w_sched, w_wire = time_sharded(args, layout, tdt, wdt, args.population, dev, rank,
                                                 args.steps, args.warmup)
            w_bytes = args.population * world * P * torch.finfo(wdt).bits // 8
            weak = {"workers_per_gpu": args.population, "population": args.population * world,
                    "ms_per_step": round(w_ms, 4), "value": round(w_bytes / (w_ms / 1e3) / 1e9, 2),
                    "unit": "GB/s", "schedule": w_sched, "wire_bytes_per_rank": w_wire,
                    "note": "companion measurement after the timed strong-scaling steps; not the value"}
        except torch.cuda.OutOfMemoryError as e:     # the value is already measured: report, go on
            weak = {"error": f"OutOfMemoryError: {str(e)[:200]}"}
            torch.cuda.empty_cache()
        sync = None

    if rank == 0:
        bg = torch.finfo(tdt).bits // 8
        bw = torch.finfo(wdt).bits // 8
        per_elem = k_local * bw + 2 * bg + (2 * bg if args.momentum else 0)
        algo_bytes = per_elem * P                       # one launch, steady state (carried buffer)
        roofline = None
        if not sharded:
            achieved = algo_bytes / (kern_ms / 1e3) / 1e9
            traffic = None
            if os.path.exists(args.traffic_json):
                try:
                    with open(args.traffic_json) as f:
                        tj = json.load(f)
                    key = f"{args.layout}/K{k_local}/{args.theta_dtype}-{args.worker_dtype}"
                    traffic = tj.get(key, {}).get("hbm_bytes_per_launch")
                except (OSError, ValueError):
                    traffic = None
            roofline = {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBPS,
                        "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBPS, 4), "traffic": traffic,
                        "kernel": kernel_name, "kernel_ms": round(kern_ms, 4),
                        "bytes_per_elem": per_elem, "algo_bytes_per_launch": algo_bytes}
        out = {
            "metric": "GB/s of param bytes reduced per outer step (device-resident), 1/2/4/8 GPUs",
            "value": round(value, 2), "unit": "GB/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(ms_per_step, 4), "higher_is_better": True,
            "scaling": scaling, "vs_baseline": None, "dtype": "f32" if tdt == torch.float32 else "bf16",
            "data": "synthetic (theta ~ N(0,.02^2), worker = theta + N(0,1e-3^2), seeded on device)",
            "config": {"workload": f"DiLoCo outer step, {args.layout} P={P} T={len(layout)}, "
                                   f"population {k_total} ({k_local} {args.worker_dtype} workers resident per GPU), "
                                   f"{args.theta_dtype} theta+momentum, lr {args.lr} mu {args.momentum} "
                                   f"nesterov {bool(args.nesterov)}",
                       "params": P, "tensors": len(layout), "workers_per_gpu": k_local,
                       "population": k_total, "worker_dtype": args.worker_dtype,
                       "theta_dtype": args.theta_dtype,
                       "parallelism": "single GPU" if not sharded else
                                       f"dp{world} {sched} (RCCL)"},
        }
        if sharded:
            # the exchange dominates: bytes this rank puts on xGMI per step over the whole step time
            # (the local HBM pass is inside that time), against the outbound direction of the
            # rank's links to its N-1 peers (it receives as much at the same time)
            wire = wire_main
            achieved = wire / (ms_per_step / 1e3) / 1e9
            peak = XGMI_LINK_GBPS * (world - 1)
            roofline = {"bound": "xgmi", "achieved": round(achieved, 1), "peak": peak, "unit": "GB/s",
                        "frac": round(achieved / peak, 4) if peak else None, "traffic": None,
                        "wire_bytes_per_rank": wire,
                        "schedule": sched}
        if roofline:
            out["roofline"] = roofline
        if weak:
            out["weak_scaling"] = weak
        if not sharded:   # what a plain device-to-device copy reaches on this device, same process
            src = torch.empty(1 << 29, dtype=torch.float32, device=dev)
            dst = torch.empty_like(src)
            dst.copy_(src)
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            for _ in range(5):
                dst.copy_(src)
            b.record()
            torch.cuda.synchronize()
            roofline["device_copy_GBps"] = round(5 * 2 * src.numel() * 4 / (a.elapsed_time(b) / 1e3) / 1e9, 1)
            del src, dst
            # the step's own access pattern with a trivial body (edt_probe_stream), same arenas:
            # the memory-system ceiling of this step on this device, measured after the timed steps
            try:
                probe_ms = stream_ceiling_ms(theta.flat, [w.flat for w in workers], sync.state.momentum)
            except Exception as e:      # a measurement extra: the JSON line still prints
                probe_ms = None
                roofline["stream_ceiling_error"] = f"{type(e).__name__}: {e}"
            if probe_ms:
                ceil = algo_bytes / (probe_ms / 1e3) / 1e9
                roofline["stream_ceiling_GBps"] = round(ceil, 1)
                roofline["frac_of_stream_ceiling"] = round(roofline["achieved"] / ceil, 4)
            if placement:
                roofline["momentum_placement"] = placement
        prop = torch.cuda.get_device_properties(dev)
        out["device"] = {"name": prop.name, "arch": getattr(prop, "gcnArchName", ""),
                         "cus": prop.multi_processor_count, "hbm_gib": round(prop.total_memory / 2**30, 1)}
        if not sharded and args.cpu_baseline_seconds > 0:
            out["cpu_baseline"] = cpu_baseline(args, tdt, wdt, k_local)
        print(json.dumps(out), flush=True)
    if sharded:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
