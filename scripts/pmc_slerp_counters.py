"""Summarise scripts/pmc_slerp_counters.sh: per kernel (lerp, speculative pass, two-pass stats and
blend) the median of every counter over its launches, plus the ratios the verdict asked for —
waves per CU and occupancy (SQ_WAVE_CYCLES counts quad-cycles, summed over the chip: x4; GRBM_GUI_ACTIVE
is summed over the 8 XCDs: / 8 is the kernel's cycles — lerp's 1.17e8 over its 7.0 ms = 8 x 2.1 GHz),
the share of wave time parked (SQ_WAIT_ANY) vs issuing, and write combining (64-B write requests
of all write requests at the memory side).

    python scripts/pmc_slerp_counters.py gpurun_out/<tag>/counters [pair|pop]
"""
import csv
import glob
import json
import os
import statistics
import sys

KERNEL_SETS = {
    "pair": {"lerp": "lerp_kernel<1, 1, 1, 8>", "speculative": "pair_sums_kernel<1, true, 1>",
             "stats": "pair_sums_kernel<1, false", "blend": "slerp_blend_tile_kernel<1, 1, true>",
             "tree_reduce": "tree_reduce_kernel"},
    # r4: BASELINE configs[4]'s population passes (scripts/pmc_pop_counters.sh)
    "pop": {"gram": "slerp_gram_kernel<1, 8>", "blend_mm": "slerp_blend_mm_kernel<1, 1, 8>",
            "pop_speculative": "slerp_pop_stats_lerp_kernel<1, 1>",
            "ring_stats": "slerp_gram_kernel<1, 8, true, false", "ring_emit": "slerp_gram_kernel<1, 8, true, true",
            "ring_emit_m2": "slerp_gram_kernel<1, 2, true, true", "triangle_m2": "slerp_gram_kernel<1, 2, false"},
    # r5: the needed-sums passes (scripts/pmc_need_counters.sh), per member count
    "need": {**{f"need_stats_d{d}": f"slerp_need_kernel<1, {d}, false" for d in range(2, 9)},
             **{f"need_emit_d{d}": f"slerp_need_kernel<1, {d}, true" for d in range(2, 9)},
             "blend_mm": "slerp_blend_mm_kernel<1, 1, "},
}
KERNELS = KERNEL_SETS["pair"]
CUS = 256
XCDS = 8


def main():
    root = sys.argv[1]
    kernels = KERNEL_SETS[sys.argv[2]] if len(sys.argv) > 2 else KERNELS
    vals = {k: {} for k in kernels}
    for path in glob.glob(os.path.join(root, "*", "**", "*counter_collection.csv"), recursive=True):
        with open(path) as f:
            for row in csv.DictReader(f):
                name = row.get("Kernel_Name", "")
                for k, sub in kernels.items():
                    if sub in name:
                        vals[k].setdefault(row["Counter_Name"], []).append(float(row["Counter_Value"]))
    out = {}
    for k, cs in vals.items():
        med = {c: statistics.median(v) for c, v in cs.items()}
        rec = {"launches": max((len(v) for v in cs.values()), default=0), "counters": med}
        g = med.get("GRBM_GUI_ACTIVE")
        if g and "SQ_WAVE_CYCLES" in med:
            cyc = g / XCDS
            rec["mean_waves_per_cu"] = round(4 * med["SQ_WAVE_CYCLES"] / cyc / CUS, 2)
            rec["occupancy_of_32_waves_per_cu"] = round(4 * med["SQ_WAVE_CYCLES"] / cyc / CUS / 32, 3)
        if "SQ_WAVE_CYCLES" in med and "SQ_WAIT_ANY" in med:
            rec["wave_time_parked"] = round(med["SQ_WAIT_ANY"] / med["SQ_WAVE_CYCLES"], 3)
            rec["wave_time_issuing"] = round(med.get("SQ_ACTIVE_INST_ANY", 0) / med["SQ_WAVE_CYCLES"], 3)
        if g and "SQ_ACTIVE_INST_VALU" in med:          # rocprof's VALUBusy: x4 / SIMDs / GUI cycles
            rec["valu_busy"] = round(med["SQ_ACTIVE_INST_VALU"] * 4 / (CUS * 4) / (g / XCDS), 3)
        if med.get("TCC_EA0_WRREQ_sum"):
            rec["write_requests_64B_share"] = round(med.get("TCC_EA0_WRREQ_64B_sum", 0) / med["TCC_EA0_WRREQ_sum"], 3)
        out[k] = rec
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from evolutionarydistributedtraining_amd._lib import library_sha256
    print(json.dumps({"probe": "pmc_slerp_counters", "lib_sha256": library_sha256(), "kernels": out}, indent=1))


if __name__ == "__main__":
    main()
