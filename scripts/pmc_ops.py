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
    # r5: the EDT-LM generation on rank-selected pairs (bench_lm_population): one launch per call,
    # the drawn generations' calls together (their floors differ: the mean floor is in the line)
    lm = traffic("pair_population_kernel")
    if lm:
        lm.update(correction="FETCH_SIZE x2 (16 B/lane bf16 loads), WRITE_SIZE x1",
                  note="per generation, median over the drawn generations' calls")
        out["lm_population/gpt_1p3b/rank"] = lm
    # r5: the drop-in tensor-list step (bench_list_form): fp32, then bf16 without and with the
    # tail masks — one template for both bf16 runs, so its launches are split in dispatch order
    import csv
    import glob

    def ordered(counter, sub):
        rows = []
        for path in glob.glob(os.path.join(root, counter, "**", "*counter_collection.csv"), recursive=True):
            with open(path) as fh:
                for row in csv.DictReader(fh):
                    if sub in row.get("Kernel_Name", "") and row.get("Counter_Name") == counter:
                        rows.append((int(row.get("Dispatch_Id") or 0), float(row["Counter_Value"])))
        return [v for _, v in sorted(rows)]

    for key, sub, part, bpe in (("f32", "outer_list_kernel<0, 0, 8", None, 48), ("bf16", "outer_list_kernel<1, 1, 8", 0, 24),
                                ("bf16_cpu_tails", "outer_list_kernel<1, 1, 8", 1, 24.125)):
        fs, ws = ordered("FETCH_SIZE", sub), ordered("WRITE_SIZE", sub)
        if part is not None:
            fs, ws = fs[part * len(fs) // 2:(part + 1) * len(fs) // 2], ws[part * len(ws) // 2:(part + 1) * len(ws) // 2]
        if not fs or not ws:
            continue
        f, w = statistics.median(fs), statistics.median(ws)
        out[f"list_form/gpt_1p3b/K8/{key}"] = {
            "kernel": sub, "launches": min(len(fs), len(ws)), "fetch_bytes_x2": 2 * f * 1024, "write_bytes": w * 1024,
            "hbm_bytes_per_launch": int(2 * f * 1024 + w * 1024), "algorithmic_bytes": int(bpe * P1),
            "correction": "FETCH_SIZE x2 (16 B/lane loads), WRITE_SIZE x1"}
    from evolutionarydistributedtraining_amd._lib import library_sha256
    for rec in out.values():
        rec["lib_sha256"] = library_sha256()      # the build these counters were measured on
    with open(os.path.join(root, "pmc_ops_traffic.json"), "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
