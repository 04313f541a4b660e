"""Summarise the PMC passes of scripts/profile_pmc.sh into per-launch HBM bytes for the fused
outer-step kernel, with the gfx950 corrections of MI355X_MICROARCH.md (HBM section):
  FETCH_SIZE (KiB) reports 1/2 of a 16-B-per-lane streaming read -> x2;  WRITE_SIZE (KiB) exact.
Access shapes other than 16 contiguous bytes per lane are uncalibrated (the guide's words): the
fp32 operands load 2 x 16 B per lane, 32 B apart. So the fetch is also calibrated on
edt_probe_stream, which bench.py runs in the same process after the timed steps: the step's exact
loads with a trivial body, each byte read once, i.e. a kernel whose read bytes are known.
  hbm_bytes_per_launch = FETCH(outer) / FETCH(probe) x known probe reads + WRITE(outer)
Writes gpurun_out/pmc/pmc_traffic.json (merge it into profiles/pmc_traffic.json for bench.py)."""
import csv
import glob
import json
import os
import statistics
import sys


def counter_values(root, counter, kernel_sub):
    vals = []
    for path in glob.glob(os.path.join(root, counter, "**", "*counter_collection.csv"), recursive=True):
        with open(path) as f:
            for row in csv.DictReader(f):
                if kernel_sub in row.get("Kernel_Name", "") and row.get("Counter_Name") == counter:
                    vals.append(float(row["Counter_Value"]))
    return vals


def main():
    root = sys.argv[1]
    extra = sys.argv[2:]
    layout, k, tdt, wdt = "gpt_1p3b", 8, "f32", "f32"          # bench.py's defaults
    for i, a in enumerate(extra):
        if a == "--layout":
            layout = extra[i + 1]
        if a == "--workers-per-gpu":
            k = int(extra[i + 1])
        if a == "--theta-dtype":
            tdt = extra[i + 1]
        if a == "--worker-dtype":
            wdt = extra[i + 1]
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from evolutionarydistributedtraining_amd.layouts import LAYOUTS
    P = LAYOUTS[layout]().total
    bw, bg = (2 if wdt == "bf16" else 4), (2 if tdt == "bf16" else 4)
    reads = (k * bw + 2 * bg) * P                 # steady state: workers, theta, momentum
    fetch = counter_values(root, "FETCH_SIZE", "outer_kernel")
    write = counter_values(root, "WRITE_SIZE", "outer_kernel")
    pfetch = counter_values(root, "FETCH_SIZE", "probe_kernel")
    # steady-state launches carry the momentum buffer: drop the first (first-step) launch
    fetch_ss, write_ss = fetch[1:] or fetch, write[1:] or write
    f_kib = statistics.median(fetch_ss)
    w_kib = statistics.median(write_ss)
    rec = {"launches": len(fetch), "fetch_kib_raw": f_kib, "write_kib": w_kib,
           "fetch_bytes_x2": 2 * f_kib * 1024, "write_bytes": w_kib * 1024,
           "algorithmic_read_bytes": reads, "algorithmic_write_bytes": 2 * bg * P}
    if pfetch:
        p_kib = statistics.median(pfetch)
        rec["probe_fetch_kib_raw"] = p_kib
        rec["fetch_over_probe"] = f_kib / p_kib
        rec["hbm_bytes_per_launch"] = int(f_kib / p_kib * reads + w_kib * 1024)
        rec["correction"] = ("fetch calibrated on edt_probe_stream (same loads, known bytes); "
                             "WRITE_SIZE x1; KiB -> bytes")
    else:
        rec["hbm_bytes_per_launch"] = int(2 * f_kib * 1024 + w_kib * 1024)
        rec["correction"] = "FETCH_SIZE x2 (gfx950 16B/lane streaming read), WRITE_SIZE x1; KiB -> bytes"
    from evolutionarydistributedtraining_amd._lib import library_sha256
    rec["lib_sha256"] = library_sha256()          # the build these counters were measured on
    out = {f"{layout}/K{k}/{tdt}-{wdt}": rec}
    with open(os.path.join(root, "pmc_traffic.json"), "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
