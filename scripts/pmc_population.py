"""HBM bytes per call of the two population-SLERP forms in bench.py's N = 1 `population_slerp_7b`
sub-object (8 x 7B members resident, 8 children), from a FETCH_SIZE and a WRITE_SIZE
rocprofv3 --pmc pass over `bench.py --ops population_7b` (scripts/profile_pmc_pop.sh): every launch
of each form's kernels summed (FETCH_SIZE x 2 and KiB -> bytes: the gfx950 corrections of
MI355X_MICROARCH.md) and divided by the calls the sub-object makes (1 warm-up + 3 timed per form).
Writes ROOT/pmc_pop_traffic.json with entries `population_7b/speculative` and
`population_7b/two_pass`, stamped with the library's sha256 (merge with scripts/merge_pmc.py).

    python scripts/pmc_population.py gpurun_out/pmc_pop
"""
import csv
import glob
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

CALLS = 4                                      # bench_population_resident: _event_ms(fn, 3, 1) per form
FORMS = {   # the kernels each form launches (tree_reduce / coef: both forms, a few MB: left out)
    "speculative": ("slerp_pop_stats_lerp_kernel", "slerp_blend_population_kernel",
                    "slerp_gram_kernel (emitting ring)", "slerp_blend_mm_kernel (redo)"),
    "two_pass": ("slerp_gram_kernel", "slerp_blend_mm_kernel"),
}


def _form_starter(name):
    """The form a call starts with this kernel (dispatch order): the speculative forms begin with the
    co-located pass or the emitting ring pass (r4: slerp_gram_kernel<IDT, M, true, true, ODT>), the
    two-pass form with a non-emitting Gram / ring pass; every later launch (blends, coefficients)
    belongs to the call its starter opened — slerp_blend_mm_kernel serves both forms."""
    if name.startswith("slerp_pop_stats_lerp_kernel"):
        return "speculative"
    if name.startswith("slerp_gram_kernel<"):
        args = [a.strip() for a in name[len("slerp_gram_kernel<"):].split(">")[0].split(",")]
        return "speculative" if len(args) >= 4 and args[3] == "true" else "two_pass"
    return None


def totals(root, counter):
    """{form: summed counter} over the slerp kernels, attributed by dispatch order."""
    rows = []
    for path in glob.glob(os.path.join(root, counter, "**", "*counter_collection.csv"), recursive=True):
        with open(path) as f:
            for row in csv.DictReader(f):
                if row.get("Counter_Name") != counter:
                    continue
                name = row["Kernel_Name"].replace("(anonymous namespace)::", "").replace("void ", "")
                if "slerp" in name:
                    rows.append((int(row.get("Dispatch_Id") or 0), name, float(row["Counter_Value"])))
    out, form = {}, None
    for _, name, v in sorted(rows):
        form = _form_starter(name) or form
        if form and (name.startswith("slerp_gram_kernel") or name.startswith("slerp_blend")
                     or name.startswith("slerp_pop_stats_lerp_kernel")):
            out[form] = out.get(form, 0.0) + v
    return out


def main():
    from evolutionarydistributedtraining_amd._lib import library_sha256
    root = sys.argv[1]
    f, w = totals(root, "FETCH_SIZE"), totals(root, "WRITE_SIZE")
    res = {}
    for form, kernels in FORMS.items():
        fetch = 2 * 1024 * f.get(form, 0.0) / CALLS
        write = 1024 * w.get(form, 0.0) / CALLS
        res[f"population_7b/{form}"] = {
            "kernels": list(kernels), "calls": CALLS, "fetch_bytes_x2": fetch, "write_bytes": write,
            "hbm_bytes_per_launch": int(round(fetch + write)),
            "correction": "FETCH_SIZE x2, WRITE_SIZE x1, KiB -> bytes; per call = all launches / calls",
            "lib_sha256": library_sha256()}
    with open(os.path.join(root, "pmc_pop_traffic.json"), "w") as fo:
        json.dump(res, fo, indent=1)
    print(json.dumps({k: [v["hbm_bytes_per_launch"], v["lib_sha256"][:12]] for k, v in res.items()}))


if __name__ == "__main__":
    main()
