"""Per-launch-shape summary of a rocprofv3 kernel trace (`--kernel-trace --output-format csv`).

rocprofv3's --stats groups by kernel name only; the bench line runs the same template at several
sizes (the 1.3B step and BASELINE configs[1]'s 125M step are both outer_kernel<0,0,8,0,0,8,false>),
so its average mixes workloads. This groups the trace by (kernel name, grid size) and prints /
writes calls and average duration per group, the figure to hold against bench.py's HIP-event
kernel times.

    python scripts/trace_by_grid.py gpurun_out/prof/bench_kernel_trace.csv [out.csv] [--filter SUB,SUB]
"""
import collections
import csv
import sys


def summarise(path, subs=("outer_kernel", "outer_list_kernel", "pair_kernel", "pair_population", "slerp", "lerp_kernel", "sgd_apply")):
    groups = collections.defaultdict(list)
    with open(path) as f:
        for r in csv.DictReader(f):
            name = r["Kernel_Name"]
            if subs and not any(s in name for s in subs):
                continue
            grid = int(r["Grid_Size_X"]) * int(r["Grid_Size_Y"]) * int(r["Grid_Size_Z"])
            groups[(name, grid)].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    rows = []
    for (name, grid), ds in sorted(groups.items(), key=lambda kv: -sum(kv[1])):
        ds.sort()
        rows.append({"kernel": name, "grid_threads": grid, "calls": len(ds),
                     "avg_ms": round(sum(ds) / len(ds) / 1e6, 4), "median_ms": round(ds[len(ds) // 2] / 1e6, 4),
                     "min_ms": round(ds[0] / 1e6, 4), "max_ms": round(ds[-1] / 1e6, 4)})
    return rows


def main():
    args = [a for a in sys.argv[1:] if not a.startswith("--filter")]
    subs = None
    for a in sys.argv[1:]:
        if a.startswith("--filter="):
            subs = tuple(a.split("=", 1)[1].split(","))
    rows = summarise(args[0], subs) if subs else summarise(args[0])
    for r in rows:
        print(f"{r['avg_ms']:10.4f} ms avg  {r['calls']:4d} calls  grid {r['grid_threads']:>10d}  {r['kernel'][:110]}")
    if len(args) > 1:
        with open(args[1], "w", newline="") as f:
            w = csv.DictWriter(f, fieldnames=list(rows[0]))
            w.writeheader()
            w.writerows(rows)


if __name__ == "__main__":
    main()
