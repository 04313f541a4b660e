"""HBM bytes per launch of the bench line's other kernels (pair_merge, slerp_7b) from the PMC
passes of scripts/profile_pmc_ops.sh, with the gfx950 corrections of MI355X_MICROARCH.md (HBM):
FETCH_SIZE (KiB) reports 1/2 of a 16-B-per-lane streaming read (these kernels load bf16 x 8 =
16 B per lane) -> x2; WRITE_SIZE exact. Merged into profiles/pmc_traffic.json under
"pair_merge/..." and "slerp_7b/..." for bench.py's sub-objects.

    python scripts/pmc_ops.py gpurun_out/pmc_ops
"""
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from pmc_summary import counter_values  # noqa: E402


def med(root, counter, name):
    v = counter_values(root, counter, name)
    return (statistics.median(v), len(v)) if v else (None, 0)


def main():
    root = sys.argv[1]
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from evolutionarydistributedtraining_amd.layouts import gpt_1p3b, qwen2p5_7b_body
    P1, P7 = gpt_1p3b().total, qwen2p5_7b_body().total
    out = {}

    def traffic(name):
        f, nf = med(root, "FETCH_SIZE", name)
        w, nw = med(root, "WRITE_SIZE", name)
        if f is None or w is None:
            return None
        return {"kernel": name, "launches": min(nf, nw), "fetch_bytes_x2": 2 * f * 1024, "write_bytes": w * 1024,
                "hbm_bytes_per_launch": int(2 * f * 1024 + w * 1024)}

    pm = traffic("pair_kernel")
    if pm:
        pm.update(algorithmic_bytes=14 * P1, correction="FETCH_SIZE x2 (16 B/lane bf16 loads), WRITE_SIZE x1")
        out["pair_merge/gpt_1p3b/bf16"] = pm
    spec = traffic("pair_sums_kernel<1, true")
    stats = traffic("pair_sums_kernel<1, false")
    blend = traffic("slerp_blend_tile_kernel<1, 1, true>")
    if spec:
        out["slerp_7b/lineage"] = {"passes": [spec], "hbm_bytes_per_launch": spec["hbm_bytes_per_launch"],
                                   "algorithmic_bytes": 6 * P7,
                                   "note": "speculative single pass (the redo blend skips every segment)"}
    if stats and blend:
        out["slerp_7b/far"] = {"passes": [stats, blend],
                               "hbm_bytes_per_launch": stats["hbm_bytes_per_launch"] + blend["hbm_bytes_per_launch"],
                               "algorithmic_bytes": 6 * P7, "moved_bytes": 10 * P7,
                               "note": "two-pass: chunk sums (4 B/elem read) + blend (4 B read, 2 B written)"}
    from evolutionarydistributedtraining_amd._lib import library_sha256
    for rec in out.values():
        rec["lib_sha256"] = library_sha256()      # the build these counters were measured on
    with open(os.path.join(root, "pmc_ops_traffic.json"), "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
