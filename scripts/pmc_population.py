"""HBM bytes per call of the two population-SLERP forms in bench.py's N = 1 `population_slerp_7b`
sub-object (8 x 7B members resident, 8 children), from a FETCH_SIZE and a WRITE_SIZE
rocprofv3 --pmc pass over `bench.py --ops population_7b` (scripts/profile_pmc_pop.sh): every launch
of each form's kernels summed (FETCH_SIZE x 2 and KiB -> bytes: the gfx950 corrections of
MI355X_MICROARCH.md) and divided by the calls (dispatch order: a call opens at its first pass).
Writes ROOT/pmc_pop_traffic.json with entries `population_7b/{roulette,ring}/{speculative,two_pass}`
(per generation), stamped with the library's sha256 (merge with scripts/merge_pmc.py).

    python scripts/pmc_population.py gpurun_out/pmc_pop
"""
import csv
import glob
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

# r5: bench_population_resident times G roulette-drawn generations then the ring of children, each
# form 1 warm-up + R timed calls (--population-generations / --population-reps; the defaults below
# must match the command in profile_pmc_pop.sh)
GENERATIONS = int(os.environ.get("POP_GENERATIONS", 3))
REPS = int(os.environ.get("POP_REPS", 10))
STARTERS = ("slerp_need_kernel", "slerp_gram_kernel", "slerp_pop_stats_lerp_kernel")
COUNTED = STARTERS + ("slerp_blend_mm_kernel", "slerp_blend_population_kernel")


def _form_of(name):
    """The form a starter kernel opens: the emitting needed-sums pass (slerp_need_kernel<IDT, D,
    true, ODT>) and the co-located pass are the speculative form's; a non-emitting needed-sums or
    triangle Gram pass the two-pass form's."""
    if name.startswith("slerp_pop_stats_lerp_kernel"):
        return "speculative"
    if name.startswith("slerp_need_kernel<"):
        args = [x.strip() for x in name[len("slerp_need_kernel<"):].split(">")[0].split(",")]
        return "speculative" if len(args) >= 3 and args[2] == "true" else "two_pass"
    return "two_pass"


def calls(root, counter):
    """[(form, summed counter)] per population call, in dispatch order: a call opens at the first
    starter kernel after a blend (a component's passes of one call follow each other)."""
    rows = []
    for path in glob.glob(os.path.join(root, counter, "**", "*counter_collection.csv"), recursive=True):
        with open(path) as f:
            for row in csv.DictReader(f):
                if row.get("Counter_Name") != counter:
                    continue
                name = row["Kernel_Name"].replace("(anonymous namespace)::", "").replace("void ", "")
                if name.startswith(COUNTED):
                    rows.append((int(row.get("Dispatch_Id") or 0), name, float(row["Counter_Value"])))
    out, prev_blend = [], True
    for _, name, v in sorted(rows):
        starter = name.startswith(STARTERS)
        if starter and prev_blend:
            out.append([_form_of(name), 0.0])
        prev_blend = not starter
        if out:
            out[-1][1] += v
    return out


def main():
    from evolutionarydistributedtraining_amd._lib import library_sha256
    root = sys.argv[1]
    f, w = calls(root, "FETCH_SIZE"), calls(root, "WRITE_SIZE")
    n_roulette = GENERATIONS * 2 * (1 + REPS)
    res = {}
    for tag, lo, hi in (("roulette", 0, n_roulette), ("ring", n_roulette, n_roulette + 2 * (1 + REPS))):
        for form in ("speculative", "two_pass"):
            fs = [v for fm, v in f[lo:hi] if fm == form]
            ws = [v for fm, v in w[lo:hi] if fm == form]
            if not fs or not ws:
                continue
            fetch = 2 * 1024 * sum(fs) / len(fs)
            write = 1024 * sum(ws) / len(ws)
            res[f"population_7b/{tag}/{form}"] = {
                "calls": len(fs), "fetch_bytes_x2": fetch, "write_bytes": write,
                "hbm_bytes_per_launch": int(round(fetch + write)),
                "note": "per call (a generation); roulette: the mean over the drawn generations",
                "correction": "FETCH_SIZE x2, WRITE_SIZE x1, KiB -> bytes",
                "lib_sha256": library_sha256()}
    with open(os.path.join(root, "pmc_pop_traffic.json"), "w") as fo:
        json.dump(res, fo, indent=1)
    print(json.dumps({k: [v["hbm_bytes_per_launch"], v["calls"], v["lib_sha256"][:12]] for k, v in res.items()}))


if __name__ == "__main__":
    main()
