"""Do reloaded parameter lists land where the previous generation's were? The drop-in DiLoCo master
reloads its base and trained models every generation (EDT_LM/diloco.py:231-235); here 292 tensors
of the 1.3B layout per model (theta + 8 workers, fp32) are freed and allocated again each
generation, in the reference's order (the previous generation's models dropped before the new ones
load: `--keep-old` loads first), and diloco.outer_step runs on them with the momentum kept in its
OuterState. Per generation: the share of theta tensors whose address repeats generation 0's, and
the step's HIP-event time — whether a momentum placement chosen once could hold.

    python scripts/list_reload_probe.py [--generations 5] [--keep-old]
"""
import argparse
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--generations", type=int, default=5)
    ap.add_argument("--keep-old", action="store_true")
    a = ap.parse_args()
    from evolutionarydistributedtraining_amd import diloco
    from evolutionarydistributedtraining_amd.layouts import gpt_1p3b
    dev = torch.device("cuda:0")
    lay = gpt_1p3b()
    K = 8
    g = torch.Generator(device=dev).manual_seed(5)

    def load():
        th = [(torch.randn(s, generator=g, device=dev) * 0.02) for s in lay.shapes]
        ws = [[t + torch.randn(t.shape, generator=g, device=dev) * 1e-3 for t in th] for _ in range(K)]
        return th, ws

    state = diloco.OuterState()
    first, out = None, []
    th = ws = None
    for gen in range(a.generations):
        if not a.keep_old:
            th = ws = None                       # the previous generation's models dropped first
        new = load()
        th, ws = new
        ptrs = [t.data_ptr() for t in th]
        first = first or ptrs
        same = sum(p == q for p, q in zip(ptrs, first)) / len(ptrs)
        diloco.outer_step(th, ws, state)         # the generation's step (creates the momentum at gen 0)
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(5)]
        for s, e in ev:
            s.record()
            diloco.outer_step(th, ws, state)
            e.record()
        torch.cuda.synchronize()
        ms = statistics.median(s.elapsed_time(e) for s, e in ev)
        out.append({"generation": gen, "theta_addresses_as_gen0": round(same, 4), "step_ms": round(ms, 4),
                    "momentum_ptr_same": state.momentum.data_ptr()})
        print(json.dumps(out[-1]), flush=True)
    print(json.dumps({"probe": "list_reload", "keep_old": a.keep_old, "generations": out}))


if __name__ == "__main__":
    main()
