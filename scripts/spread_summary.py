"""Tabulate scripts/gpu_r6_spread.sh's lines (gpurun_out/spread/*.json): per process the headline's
placed and first-allocation figures, the whole-set draws, and configs[1]'s pair; then a summary.

    python scripts/spread_summary.py gpurun_out/spread > profiles/r06_spread.jsonl
"""
import glob
import json
import os
import sys


def main(d):
    rows = []
    for path in sorted(glob.glob(os.path.join(d, "*.json"))):
        if path.endswith("_detail.json"):
            continue
        with open(path) as f:
            line = json.load(f)
        r, c = line["roofline"], line.get("configs1_125m", {})
        rows.append({"run": os.path.basename(path)[:-5], "kernel_ms": r["kernel_ms"], "frac": r["frac"],
                     "unplaced_ms": r.get("unplaced_ms"), "unplaced_frac": r.get("unplaced_frac"),
                     "draws_ms": r.get("placement", {}).get("draws_ms"),
                     "chosen_draw": r.get("placement", {}).get("chosen_draw"),
                     "configs1_frac": c.get("roofline", {}).get("frac"), "configs1_unplaced_frac": c.get("unplaced_frac"),
                     "configs1_draws_ms": c.get("placement", {}).get("draws_ms"),
                     "lib": line.get("native", {}).get("sha256", "")[:12]})
    for row in rows:
        print(json.dumps(row))

    def span(key):
        v = [row[key] for row in rows if row[key] is not None]
        return [min(v), max(v)] if v else None
    first_draw_best = [min(row["draws_ms"][:1]) for row in rows if row["draws_ms"]]
    print(json.dumps({"summary": True, "processes": len(rows), "frac": span("frac"),
                      "unplaced_frac": span("unplaced_frac"), "configs1_frac": span("configs1_frac"),
                      "configs1_unplaced_frac": span("configs1_unplaced_frac"),
                      "chosen_draw_not_first": sum(1 for row in rows if row["chosen_draw"]),
                      "gain_over_first_draw_ms": [round(f - row["kernel_ms"], 4) for f, row in
                                                  zip(first_draw_best, rows)]}))


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/spread")
