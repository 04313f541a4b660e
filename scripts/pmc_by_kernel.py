"""Median FETCH_SIZE x2 / WRITE_SIZE (bytes, gfx950 corrections of MI355X_MICROARCH.md) per kernel
name over every launch in a pair of rocprofv3 --pmc passes (ROOT/FETCH_SIZE, ROOT/WRITE_SIZE).

    python scripts/pmc_by_kernel.py gpurun_out/<tag>/pmc
"""
import csv
import glob
import json
import os
import statistics
import sys


def per_kernel(root, counter):
    vals = {}
    for path in glob.glob(os.path.join(root, counter, "**", "*counter_collection.csv"), recursive=True):
        with open(path) as f:
            for row in csv.DictReader(f):
                if row.get("Counter_Name") == counter:
                    name = row["Kernel_Name"].replace("(anonymous namespace)::", "").replace("void ", "")
                    name = name.split("(")[0]
                    vals.setdefault(name[:90], []).append(float(row["Counter_Value"]))
    return vals


def main():
    root = sys.argv[1]
    f, w = per_kernel(root, "FETCH_SIZE"), per_kernel(root, "WRITE_SIZE")
    out = {}
    for k in sorted(set(f) | set(w)):
        out[k] = {"launches": len(f.get(k, [])),
                  "fetch_bytes_x2_median": 2 * 1024 * statistics.median(f[k]) if k in f else None,
                  "write_bytes_median": 1024 * statistics.median(w[k]) if k in w else None,
                  "fetch_bytes_x2_all": [round(2 * 1024 * v) for v in f.get(k, [])]}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
