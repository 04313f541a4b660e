"""The checkpoint edge at the north star's sizes: safetensors
files -> pinned host -> HBM -> kernel -> files, as the reference's master does it through its shared
disk (EDT_LM/diloco.py:231-235 gather, :302-308 broadcast; EDT_EVOMERGE/train/crossover.py:86-146).

  diloco  1.3B x 8 bf16 worker checkpoints + the bf16 base: checkpoint.read_many (one reader
          thread + pinned staging + copy stream per checkpoint) -> fused outer step ->
          checkpoint.save_to_dirs (one D2H, then the 8 files written in parallel, in place of the
          workers' as DirOuterSync does); then DirOuterSync.step end to end on the same dirs.
  slerp   one SLERP child of two 7.07B bf16 bodies: both parents read into arenas -> slerp_arena
          -> the child written (write_from_arena).
Files go to a scratch dir (page cache warm after writing: the best case of a shared disk) and are
deleted at the end. Rates are of the files' bytes. Before each timed phase the page cache's dirty
pages are flushed (os.sync(), untimed, its duration reported): otherwise a write phase pays for the
write-back of the files created just before it, and the figures track the file system's flusher,
not the path.

    python scripts/e2e_checkpoint_large.py --dir /path/with/80GB
"""
from __future__ import annotations

import argparse
import json
import os
import shutil
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def _fill(flat, seed, base=None, scale=0.02):
    g = torch.Generator(device=flat.device).manual_seed(seed)
    step = 1 << 28
    for s in range(0, flat.numel(), step):
        e = min(flat.numel(), s + step)
        x = torch.randn(e - s, generator=g, device=flat.device) * scale
        if base is not None:
            x += base[s:e].float()
        flat[s:e] = x.to(flat.dtype)


SYNCS = []


def _sync_time(fn):
    t0 = time.perf_counter()
    os.sync()                     # untimed: flush the dirty pages earlier phases left
    SYNCS.append(round(time.perf_counter() - t0, 2))
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    out = fn()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    print(f"  phase done in {dt:.2f} s", file=sys.stderr, flush=True)     # progress for long runs
    return dt, out


def diloco(a, dev, root):
    from evolutionarydistributedtraining_amd import checkpoint, ops
    from evolutionarydistributedtraining_amd.diloco import DirOuterSync
    from evolutionarydistributedtraining_amd.layouts import gpt_1p3b
    lay = gpt_1p3b()
    P, bf = lay.total, torch.bfloat16
    base_dir = os.path.join(root, "base")
    wdirs = [os.path.join(root, f"w{k}") for k in range(a.k)]
    theta = torch.empty(P, dtype=bf, device=dev)
    _fill(theta, 1)
    os.makedirs(base_dir, exist_ok=True)
    checkpoint.write_from_arena(os.path.join(base_dir, "model.safetensors"), lay, theta)
    tmp = torch.empty_like(theta)
    for k, d in enumerate(wdirs):
        _fill(tmp, 10 + k, base=theta, scale=1e-3)
        os.makedirs(d, exist_ok=True)
        checkpoint.write_from_arena(os.path.join(d, "model.safetensors"), lay, tmp)
        print(f"  wrote worker {k}", file=sys.stderr, flush=True)
    del tmp
    file_bytes = (a.k + 1) * P * 2
    workers = [torch.empty(P, dtype=bf, device=dev) for _ in range(a.k)]
    mom = torch.zeros(P, dtype=bf, device=dev)
    res = {"layout": "gpt_1p3b", "P": P, "K": a.k, "dtype": "bf16", "files_read_bytes": file_bytes,
           "files_written_bytes": a.k * P * 2}
    t_read, _ = _sync_time(lambda: checkpoint.read_many([(base_dir, theta)] + list(zip(wdirs, workers)), lay))
    t_step, _ = _sync_time(lambda: ops.outer_step(theta, workers, mom, False, 0.7, 0.9, True))
    t_write, _ = _sync_time(lambda: checkpoint.save_to_dirs(wdirs, lay, theta))
    res["phases"] = {"read_ms": round(t_read * 1e3, 1), "read_GBps": round(file_bytes / t_read / 1e9, 2),
                     "step_ms": round(t_step * 1e3, 2), "write_ms": round(t_write * 1e3, 1),
                     "write_GBps": round(a.k * P * 2 / t_write / 1e9, 2),
                     "total_ms": round((t_read + t_step + t_write) * 1e3, 1)}
    del workers, mom, theta
    torch.cuda.empty_cache()
    # DirOuterSync end to end (generation 1: base + workers read; generation 2: theta resident)
    sync = DirOuterSync(device=dev, names=lay.names, place_draws=a.place_draws)
    t1, _ = _sync_time(lambda: sync.step(base_dir, wdirs))
    t2, _ = _sync_time(lambda: sync.step(wdirs[0], wdirs))
    t3, _ = _sync_time(lambda: sync.step(wdirs[0], wdirs))
    pl = sync.placement or {}
    res["dir_outer_sync"] = {"generation_ms": round(t1 * 1e3, 1), "resident_theta_generation_ms": round(t2 * 1e3, 1),
                             "third_generation_ms": round(t3 * 1e3, 1),
                             "metric_GBps_e2e": round(a.k * P * 2 / t2 / 1e9, 2),
                             "placement": {"seconds": pl.get("seconds"), "place_draws": a.place_draws,
                                           "draws_ms": [d["best_ms"] for d in pl.get("draws", [])]}}
    del sync
    torch.cuda.empty_cache()
    for d in [base_dir] + wdirs:
        shutil.rmtree(d, ignore_errors=True)
    return res


def slerp(a, dev, root):
    from evolutionarydistributedtraining_amd import checkpoint, ops
    from evolutionarydistributedtraining_amd.layouts import qwen2p5_7b_body
    lay = qwen2p5_7b_body()
    P, bf = lay.total, torch.bfloat16
    dirs = [os.path.join(root, f"parent{i}") for i in range(2)]
    v0 = torch.empty(P, dtype=bf, device=dev)
    v1 = torch.empty(P, dtype=bf, device=dev)
    _fill(v0, 3)
    _fill(v1, 4, base=v0, scale=1e-3)
    for d, v in zip(dirs, (v0, v1)):
        os.makedirs(d, exist_ok=True)
        checkpoint.write_from_arena(os.path.join(d, "model.safetensors"), lay, v)
    out = torch.empty(P, dtype=bf, device=dev)
    plan = ops.make_slerp_plan(lay.offsets, dev)
    t = torch.full((len(lay),), 0.5, dtype=torch.float64, device=dev)
    ops.slerp_arena(plan, v0, v1, out, t)          # warm the plan (two-pass chosen for far parents)
    child = os.path.join(root, "child")
    os.makedirs(child, exist_ok=True)
    t_read, _ = _sync_time(lambda: checkpoint.read_many(list(zip(dirs, (v0, v1))), lay))
    t_merge, _ = _sync_time(lambda: ops.slerp_arena(plan, v0, v1, out, t))
    t_write, _ = _sync_time(lambda: checkpoint.write_from_arena(os.path.join(child, "model.safetensors"), lay, out))
    sharded = os.path.join(root, "child_sharded")
    t_shard, files = _sync_time(lambda: checkpoint.write_sharded_from_arena(sharded, lay, out, a.shard_bytes))
    res = {"layout": "qwen2p5_7b_body", "P": P, "dtype": "bf16",
           "phases": {"read_ms": round(t_read * 1e3, 1), "read_GBps": round(4 * P / t_read / 1e9, 2),
                      "merge_ms": round(t_merge * 1e3, 2), "write_ms": round(t_write * 1e3, 1),
                      "write_GBps": round(2 * P / t_write / 1e9, 2),
                      "total_ms": round((t_read + t_merge + t_write) * 1e3, 1)},
           "sharded_write": {"shard_bytes": a.shard_bytes, "shards": len(files), "ms": round(t_shard * 1e3, 1),
                             "GBps": round(2 * P / t_shard / 1e9, 2),
                             "total_ms": round((t_read + t_merge + t_shard) * 1e3, 1)}}
    back = torch.empty_like(out)                  # the shards read back equal the child
    checkpoint.read_many([(sharded, back)], lay)
    torch.cuda.synchronize()
    res["sharded_write"]["reads_back_equal"] = bool(torch.equal(back, out))
    del back
    for d in dirs + [child, sharded]:
        shutil.rmtree(d, ignore_errors=True)
    return res


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--what", default="diloco,slerp")
    ap.add_argument("--dir", default=os.path.join(os.getcwd(), "e2e_ckpt_tmp"))
    ap.add_argument("--k", type=int, default=8)
    ap.add_argument("--place-draws", type=int, default=1, help="DirOuterSync(place_draws=...)")
    ap.add_argument("--shard-bytes", type=int, default=4 << 30, help="slerp: write_sharded_from_arena's shard size")
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    os.makedirs(a.dir, exist_ok=True)
    try:
        if "diloco" in a.what:
            print(json.dumps({"diloco": diloco(a, dev, a.dir), "os_sync_s_before_phases": SYNCS[:]}), flush=True)
            SYNCS.clear()
            torch.cuda.empty_cache()
        if "slerp" in a.what:
            print(json.dumps({"slerp": slerp(a, dev, a.dir), "os_sync_s_before_phases": SYNCS[:]}), flush=True)
    finally:
        shutil.rmtree(a.dir, ignore_errors=True)


if __name__ == "__main__":
    main()
