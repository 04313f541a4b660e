"""How much of the fused step's speed is the allocation? Allocates D independent sets of the bench
operands (fp32 theta, momentum and 8 fp32 workers at 1.3B: 52.6 GB per set), all held at once so
every set gets its own physical pages, and times the product kernel (ops.outer_step) and the
stream-ceiling probe on each set, in interleaved rounds so that drift over time is visible.
Prints one JSON object.

    python scripts/alloc_draws.py [--draws 3] [--rounds 3] [--params 1315723264]
"""
from __future__ import annotations

import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bench import stream_ceiling_ms  # noqa: E402
from evolutionarydistributedtraining_amd import ops  # noqa: E402


def time_step(theta, workers, mom, iters=10):
    ops.outer_step(theta, workers, mom, True, 0.7, 0.9, True)
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(iters)]
    for a, b in ev:
        a.record()
        ops.outer_step(theta, workers, mom, True, 0.7, 0.9, True)
        b.record()
    torch.cuda.synchronize()
    ts = sorted(a.elapsed_time(b) for a, b in ev)
    return ts[len(ts) // 2]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--draws", type=int, default=3)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--params", type=int, default=1315723264)
    ap.add_argument("--workers", type=int, default=8)
    ap.add_argument("--mix", action="store_true",
                    help="also time operand sets mixed across draws (which streams carry the spread)")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    n, k = a.params, a.workers
    sets = []
    for d in range(a.draws):
        theta = torch.randn(n, device=dev) * 0.02
        mom = torch.randn(n, device=dev) * 1e-4
        workers = []
        for _ in range(k):
            w = torch.empty(n, device=dev)
            w.copy_(theta)
            workers.append(w)
        sets.append((theta, workers, mom))
        print(f"draw {d}: theta {theta.data_ptr():#x} mom {mom.data_ptr():#x} workers "
              + " ".join(f"{w.data_ptr():#x}" for w in workers), flush=True)
    algo = n * (k * 4 + 4 * 4)
    out = {"params": n, "workers": k, "algo_bytes": algo, "rounds": []}
    for r in range(a.rounds):
        row = []
        for d, (theta, workers, mom) in enumerate(sets):
            step = time_step(theta, workers, mom)
            probe = stream_ceiling_ms(theta, workers, mom)
            row.append({"draw": d, "step_ms": round(step, 4), "probe_ms": round(probe, 4),
                        "step_TBps": round(algo / step / 1e9, 3)})
            print(json.dumps(row[-1]), flush=True)
        out["rounds"].append(row)
    if a.mix and len(sets) >= 2:
        lo, hi = 0, len(sets) - 1
        h = k // 2
        combos = {
            "theta_mom_first_workers_last": (sets[lo][0], sets[hi][1], sets[lo][2]),
            "theta_mom_last_workers_first": (sets[hi][0], sets[lo][1], sets[hi][2]),
            "workers_half_first_half_last": (sets[lo][0], sets[lo][1][:h] + sets[hi][1][h:], sets[lo][2]),
            "workers_first_half_only_from_last": (sets[lo][0], sets[hi][1][:h] + sets[lo][1][h:], sets[lo][2]),
        }
        for ti in range(len(sets)):            # theta from draw ti, momentum from draw mi
            for mi in range(len(sets)):
                combos[f"theta{ti}_mom{mi}_workers0"] = (sets[ti][0], sets[lo][1], sets[mi][2])
        out["mix"] = {}
        for name, (theta, workers, mom) in combos.items():
            step = time_step(theta, workers, mom)
            out["mix"][name] = round(step, 4)
            print(name, round(step, 4), flush=True)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
