"""The timed steps' launches out of a rocprofv3 kernel trace of `python bench.py`: the fused step
template at the 1.3B grid, in launch order, is [1 first step + 4 warm-up] [5 first-allocation
(unplaced) launches] [1 after the placement search] [the --steps timed launches] [2 traced] [the
step-with-broadcast comparison] [the list_form same-memory arenas]. The whole-trace average mixes
those (other arenas, other placements); this prints the mean over the timed window and the
unplaced window, to hold against the line's roofline.kernel_ms / unplaced_ms from HIP events.

    python scripts/timed_window.py gpurun_out/r6final/bkt/bench_kernel_trace.csv [--steps 20 --warmup 5]
"""
import argparse
import csv
import json
import statistics


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--kernel", default="outer_kernel<0, 0, 8, 0, 0, 8, false>")
    ap.add_argument("--grid", type=int, default=164465408)          # 1.3B: 80,315 workgroups x 256 x 8
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    a = ap.parse_args()
    rows = [r for r in csv.DictReader(open(a.trace))
            if a.kernel in r["Kernel_Name"] and int(r["Grid_Size_X"]) * int(r["Grid_Size_Y"]) * int(r["Grid_Size_Z"]) == a.grid]
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    d = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6 for r in rows]
    un0 = a.warmup
    t0 = a.warmup + 5 + 1
    print(json.dumps({"kernel": a.kernel, "grid_threads": a.grid, "launches": len(d),
                      "timed_window": [t0, t0 + a.steps], "timed_mean_ms": round(statistics.mean(d[t0:t0 + a.steps]), 4),
                      "unplaced_window": [un0, un0 + 5], "unplaced_mean_ms": round(statistics.mean(d[un0:un0 + 5]), 4),
                      "all_mean_ms": round(statistics.mean(d), 4)}))


if __name__ == "__main__":
    main()
