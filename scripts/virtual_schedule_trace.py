"""The multi-GPU schedules on N virtual ranks in one process on one MI355X (collectives.VirtualWorld),
for a rocprofv3 --marker-trace --kernel-trace capture: the roctx ranges of the shim's phases
(tracing.py) around the HIP kernels and the device copies that stand in for the collectives.
Timings are of the virtual schedule (collectives as device copies), not of xGMI.

    python scripts/virtual_schedule_trace.py [--layout gpt2_small --world 4]
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
    ap.add_argument("--world", type=int, default=4)
    ap.add_argument("--steps", type=int, default=3)
    a = ap.parse_args()
    from evolutionarydistributedtraining_amd.collectives import VirtualWorld
    from evolutionarydistributedtraining_amd.distributed import ShardedOuterSync, ShardedPopulationCrossover
    from evolutionarydistributedtraining_amd.layouts import LAYOUTS
    dev = torch.device("cuda:0")
    lay = LAYOUTS[a.layout]()
    P, N = lay.total, a.world
    res = {"layout": a.layout, "P": P, "world": N}
    for mode, bc in (("exact", "workers"), ("reduce", "theta")):
        def body(comm):
            s = ShardedOuterSync(lay, torch.float32, torch.bfloat16, 8 // N, dev, mode=mode, broadcast=bc, comm=comm)
            g = torch.Generator(device=dev).manual_seed(comm.rank)
            s.theta.flat.copy_(torch.randn(P, generator=g, device=dev) * 0.02)
            for w in s.workers:
                w.flat.copy_(s.theta.flat + torch.randn(P, generator=g, device=dev) * 1e-3)
            for _ in range(a.steps):
                s.step()
            torch.cuda.synchronize()
            comm.barrier()
            t0 = time.perf_counter()
            for _ in range(a.steps):
                s.step()
            torch.cuda.synchronize()
            comm.barrier()
            return (time.perf_counter() - t0) / a.steps * 1e3
        ms = VirtualWorld(N).run(body)
        res[f"outer_{mode}_{bc}_ms"] = round(max(ms), 3)
    members = [(torch.randn(P, device=dev) * 0.02).bfloat16() for _ in range(N)]
    pairs = [((3 * c + 1) % N, (5 * c + 2) % N) for c in range(N)]
    t = torch.full((len(lay),), 0.5, dtype=torch.float64, device=dev)

    def pop(comm):
        sp = ShardedPopulationCrossover(lay, torch.bfloat16, dev, kind="slerp", comm=comm)
        out = torch.empty(P, dtype=torch.bfloat16, device=dev)
        for _ in range(2):
            sp.slerp_step(members[comm.rank], pairs, t, out)
        torch.cuda.synchronize()
        comm.barrier()
        t0 = time.perf_counter()
        sp.slerp_step(members[comm.rank], pairs, t, out)
        torch.cuda.synchronize()
        comm.barrier()
        return (time.perf_counter() - t0) * 1e3
    res["sharded_population_slerp_ms"] = round(max(VirtualWorld(N).run(pop)), 3)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
