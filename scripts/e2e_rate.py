"""End-to-end DiLoCo outer-step rate when the population arrives from the host (PCIe-inclusive).

In the reference the replicas come from other hosts through checkpoints on a shared disk
(EDT_LM/diloco.py:231-235) and the new global weights go back the same way (:302-308). This
measures the device side of that edge: K worker arenas in pinned host memory -> H2D -> fused
outer step -> D2H of the new theta, (a) serial and (b) bucketed, H2D of bucket b+1 on a copy
stream overlapping the kernel on bucket b. Reported as the metric (K x P x bytes / time) and as
PCIe GB/s moved. Not the bench `value` (that one is device-resident).

    python scripts/e2e_rate.py [--layout gpt2_small --k 8 --bucket-elems 16777216]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--layout", default="gpt2_small")
    ap.add_argument("--k", type=int, default=8)
    ap.add_argument("--bucket-elems", type=int, default=1 << 24)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--disk-dir", default=None, help="also time the checkpoint edge through files here")
    a = ap.parse_args()
    from evolutionarydistributedtraining_amd import ops
    from evolutionarydistributedtraining_amd.layouts import LAYOUTS
    dev = torch.device("cuda:0")
    P = LAYOUTS[a.layout]().total
    g = torch.Generator().manual_seed(0)
    theta_h = (torch.randn(P, generator=g) * 0.02).pin_memory()
    workers_h = [(theta_h + torch.randn(P, generator=g) * 1e-3).bfloat16().pin_memory() for _ in range(a.k)]
    theta_out_h = torch.empty(P, dtype=torch.float32).pin_memory()
    theta_d = torch.empty(P, device=dev)
    mom_d = torch.zeros(P, device=dev)
    workers_d = [torch.empty(P, dtype=torch.bfloat16, device=dev) for _ in range(a.k)]
    metric_bytes = a.k * P * 2
    pcie_bytes = metric_bytes + 4 * P + 4 * P     # workers + theta in, theta out

    def serial():
        theta_d.copy_(theta_h, non_blocking=True)
        for wd, wh in zip(workers_d, workers_h):
            wd.copy_(wh, non_blocking=True)
        ops.outer_step(theta_d, workers_d, mom_d, True, 0.7, 0.9, True)
        theta_out_h.copy_(theta_d, non_blocking=True)

    copy = torch.cuda.Stream(dev)
    comp = torch.cuda.current_stream(dev)

    def pipelined():
        evs = []
        B = a.bucket_elems
        for s in range(0, P, B):
            e = min(P, s + B)
            with torch.cuda.stream(copy):
                theta_d[s:e].copy_(theta_h[s:e], non_blocking=True)
                for wd, wh in zip(workers_d, workers_h):
                    wd[s:e].copy_(wh[s:e], non_blocking=True)
                ev = torch.cuda.Event()
                ev.record(copy)
            evs.append((s, e, ev))
        for s, e, ev in evs:
            comp.wait_event(ev)
            ops.outer_step(theta_d[s:e], [w[s:e] for w in workers_d], mom_d[s:e], True, 0.7, 0.9, True)
            theta_out_h[s:e].copy_(theta_d[s:e], non_blocking=True)

    res = {}
    for name, fn in (("serial", serial), ("pipelined", pipelined)):
        fn()
        torch.cuda.synchronize()
        ts = []
        for _ in range(a.reps):
            t0 = time.perf_counter()
            fn()
            torch.cuda.synchronize()
            ts.append(time.perf_counter() - t0)
        t = min(ts)
        res[name] = {"ms": round(t * 1e3, 2), "metric_GBps": round(metric_bytes / t / 1e9, 2),
                     "pcie_GBps": round(pcie_bytes / t / 1e9, 2)}
    # kernel alone, device-resident, for reference
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.reps):
        ops.outer_step(theta_d, workers_d, mom_d, True, 0.7, 0.9, True)
    torch.cuda.synchronize()
    tk = (time.perf_counter() - t0) / a.reps
    res["device_resident"] = {"ms": round(tk * 1e3, 3), "metric_GBps": round(metric_bytes / tk / 1e9, 1)}
    if a.disk_dir:
        res["checkpoint_edge"] = disk_edge(a, P, workers_h, theta_d, mom_d, workers_d, metric_bytes)
    print(json.dumps({"layout": a.layout, "P": P, "K": a.k, "bucket_elems": a.bucket_elems, **res}))


def disk_edge(a, P, workers_h, theta_d, mom_d, workers_d, metric_bytes):
    """The gather/broadcast edge through checkpoint files (EDT_LM/diloco.py:231-235, 302-308):
    K worker dirs -> arenas (checkpoint.read_into_arena) -> outer step -> new theta to K dirs
    (checkpoint.save_to_dirs), against safetensors.load_file/save_file per worker (the loader
    HF from_pretrained/save_pretrained use), page cache warm for both."""
    import shutil
    import tempfile
    from safetensors.torch import load_file, save_file
    from evolutionarydistributedtraining_amd import checkpoint, ops
    from evolutionarydistributedtraining_amd.layouts import LAYOUTS
    lay = LAYOUTS[a.layout]()
    root = tempfile.mkdtemp(dir=a.disk_dir)
    try:
        dirs = [os.path.join(root, f"w{k}") for k in range(a.k)]
        for d, wh in zip(dirs, workers_h):
            os.makedirs(d)
            checkpoint.write_from_arena(os.path.join(d, "model.safetensors"), lay, wh)
        out_dirs = [os.path.join(root, f"o{k}") for k in range(a.k)]
        out = {}
        for rep in range(2):                      # second pass: warm page cache
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            tr = time.perf_counter()
            for d, wd in zip(dirs, workers_d):
                checkpoint.read_into_arena(d, lay, wd)
            torch.cuda.synchronize()
            serial_read = time.perf_counter() - tr
            t0 = time.perf_counter()
            checkpoint.read_many(list(zip(dirs, workers_d)), lay, threads=a.k)
            torch.cuda.synchronize()
            t1 = time.perf_counter()
            ops.outer_step(theta_d, workers_d, mom_d, True, 0.7, 0.9, True)
            torch.cuda.synchronize()
            t2 = time.perf_counter()
            checkpoint.save_to_dirs(out_dirs, lay, theta_d)
            t3 = time.perf_counter()
            out = {"read_serial_ms": round(serial_read * 1e3, 1),
                   "read_ms": round((t1 - t0) * 1e3, 1), "step_ms": round((t2 - t1) * 1e3, 2),
                   "write_ms": round((t3 - t2) * 1e3, 1),
                   "read_GBps": round(metric_bytes / (t1 - t0) / 1e9, 2),
                   "total_metric_GBps": round(metric_bytes / (t3 - t0) / 1e9, 2)}
        # per-worker safetensors load/save, as from_pretrained / save_pretrained do it
        t0 = time.perf_counter()
        for d, wd in zip(dirs, workers_d):
            sd = load_file(os.path.join(d, "model.safetensors"))
            for v, n in zip(lay.views(wd), lay.names):
                v.copy_(sd[n])
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        cpu_theta = {n: v.detach().cpu().contiguous() for n, v in zip(lay.names, lay.views(theta_d))}
        for d in out_dirs:
            save_file(cpu_theta, os.path.join(d, "ref.safetensors"))
        t2 = time.perf_counter()
        out["safetensors_load_ms"] = round((t1 - t0) * 1e3, 1)
        out["safetensors_save_ms"] = round((t2 - t1) * 1e3, 1)
        return out
    finally:
        shutil.rmtree(root, ignore_errors=True)


if __name__ == "__main__":
    main()
