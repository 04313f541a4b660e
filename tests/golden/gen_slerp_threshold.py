"""Golden cases for the SLERP branch decision at the reference's DOT_THRESHOLD = 0.9995
(EDT_RL/crossover.py:24-31; EDT_EVOMERGE/train/crossover.py's copy), generated FROM THE REFERENCE.

Test infrastructure only; runs in the build container (needs /root/reference), never imported by
the tests, smoke() or bench.py. The reference's own `slerp` and `normalize` are imported by path;
only numbers are written out.

Cases: true cosine (fp64, of the rounded inputs) at 0.9995 +- {1e-7, 1e-6, 1e-5}, fp32 and bf16
inputs, a 437-element tensor (stored whole) and a 1,048,583-element one (rebuilt by the tests from
seed + noise scale, tests/golden/threshold_inputs.py; the reference output is stored at 4,096
sampled elements with an fp64 checksum of all of it). For each: the reference's fp32 dot (the value
its branch test sees), its branch, and its output at t = 0.5 (and t = 0.3 for the small cases).

    python tests/golden/gen_slerp_threshold.py
"""
from __future__ import annotations

import importlib.util
import json
import os
import sys

import numpy as np
import torch
from safetensors.torch import save_file

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
from threshold_inputs import digest, exact_cos, make_pair, sample_index  # noqa: E402

REF = "/root/reference"
THR = 0.9995


def _load(name, rel):
    spec = importlib.util.spec_from_file_location(name, os.path.join(REF, rel))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def _solve_s(seed, n, dtype, target):
    """Noise scale whose rounded pair has exact cosine ~ target (bisection; cos falls with s)."""
    lo, hi = 0.0, 0.2
    best = None
    for _ in range(60):
        mid = 0.5 * (lo + hi)
        c = exact_cos(*make_pair(seed, n, dtype, mid))
        if best is None or abs(c - target) < abs(best[1] - target):
            best = (mid, c)
        if c > target:
            lo = mid
        else:
            hi = mid
    return best


def main():
    rl = _load("ref_rl_crossover", "EDT_RL/crossover.py")
    tensors, cases = {}, []
    seed = 4242
    for size_tag, n in (("small", 437), ("large", 1_048_583)):
        for dtype in ("f32", "bf16"):
            for off in (-1e-5, -1e-6, -1e-7, 1e-7, 1e-6, 1e-5):
                seed += 1
                s, cos = _solve_s(seed, n, dtype, THR + off)
                a, b = make_pair(seed, n, dtype, s)
                dot_ref = float(np.sum(rl.normalize(a.float().numpy(), 1e-8) * rl.normalize(b.float().numpy(), 1e-8)))
                name = f"thr/{size_tag}_{dtype}_{off:+.0e}"
                rec = {"name": name, "seed": seed, "n": n, "dtype": dtype, "noise_scale": s, "target_offset": off,
                       "exact_cos": cos, "ref_dot": dot_ref, "ref_lerp_branch": bool(abs(dot_ref) > THR),
                       "exact_lerp_branch": bool(abs(cos) > THR), "sha256": digest(a, b),
                       "source": "EDT_RL/crossover.py:11-43", "outputs": []}
                if size_tag == "small":
                    tensors[f"{name}/v0"] = a.contiguous()
                    tensors[f"{name}/v1"] = b.contiguous()
                idx = sample_index(n)
                for t in ((0.5, 0.3) if size_tag == "small" else (0.5,)):
                    out = rl.slerp(t, a, b)
                    key = f"{name}/t{t}"
                    tensors[f"{key}/out"] = out[idx].contiguous()
                    rec["outputs"].append({"t": t, "key": key, "sum_f64": float(out.double().sum())})
                cases.append(rec)
                print(name, f"exact {cos:.10f} ref {dot_ref:.10f}", "straddle" if rec["ref_lerp_branch"] !=
                      rec["exact_lerp_branch"] else "")
    save_file(tensors, os.path.join(HERE, "slerp_threshold.safetensors"))
    with open(os.path.join(HERE, "slerp_threshold.json"), "w") as f:
        json.dump({"generated_with": {"torch": torch.__version__, "numpy": np.__version__},
                   "threshold": THR, "cases": cases}, f, indent=1)


if __name__ == "__main__":
    main()
