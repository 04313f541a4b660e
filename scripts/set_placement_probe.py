"""Is the headline step's placement floor a property of the whole operand set's region (as at
125M, profiles/r06_config1_joint.jsonl), so that re-drawing the whole set (θ, the K workers and the
momentum) in other regions finds better placements than the momentum search inside one draw?

Per draw d (each behind a held spacer of d x SPACER_GIB, earlier draws' θ and workers held so every
draw lands elsewhere): the probe kernel (the step's access pattern) on the first allocation, then
place_momentum's best candidate — for the 1.3B fp32 x 8 step (LAYOUT=gpt_1p3b, default) or 125M.

    python scripts/set_placement_probe.py > profiles/r06_set_placement_probe.jsonl     # GPU box
"""
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from evolutionarydistributedtraining_amd.layouts import LAYOUTS  # noqa: E402
from evolutionarydistributedtraining_amd.placement import place_momentum, probe_ms  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    P = LAYOUTS[os.environ.get("LAYOUT", "gpt_1p3b")]().total
    draws = int(os.environ.get("DRAWS", "3"))
    spacer = int(float(os.environ.get("SPACER_GIB", "7")) * (1 << 30))
    K = 8
    held = []
    res = []
    for d in range(draws):
        if d:
            held.append(torch.empty(d * spacer, dtype=torch.uint8, device=dev))
        g = torch.Generator(device=dev).manual_seed(500 + d)
        theta = torch.randn(P, generator=g, device=dev) * 0.02
        workers = [theta + torch.randn(P, generator=g, device=dev) * 1e-3 for _ in range(K)]
        mom = torch.randn(P, generator=g, device=dev) * 1e-3
        first = probe_ms(theta, workers, mom, iters=5)
        mom2, rep = place_momentum(theta, workers, mom, 8)
        best = min(rep["probe_ms"]) if rep["probe_ms"] else first
        rec = {"draw": d, "P": P, "first_ms": round(first, 4), "placed_best_ms": round(best, 4),
               "placement": rep, "free_gib_after": round(torch.cuda.mem_get_info(dev)[0] / 2**30, 1)}
        res.append(rec)
        print(json.dumps(rec), flush=True)
        del mom, mom2
        held.append((theta, workers))
        torch.cuda.empty_cache()
    print(json.dumps({"summary": True, "first_ms": [r["first_ms"] for r in res],
                      "placed_best_ms": [r["placed_best_ms"] for r in res],
                      "best_of_draws_ms": min(r["placed_best_ms"] for r in res),
                      "draw0_placed_ms": res[0]["placed_best_ms"]}), flush=True)


if __name__ == "__main__":
    main()
