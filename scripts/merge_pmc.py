"""Merge the PMC summaries of one GPU call (scripts/profile_pmc.sh -> pmc_traffic.json,
scripts/profile_pmc_ops.sh -> pmc_ops_traffic.json; every entry stamped with the library's sha256)
into profiles/pmc_traffic.json, which bench.py reads for roofline.traffic.

    python scripts/merge_pmc.py gpurun_out/pmc_X/pmc_traffic.json gpurun_out/pmc_ops/pmc_ops_traffic.json [--out F]
"""
import argparse
import json
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("summaries", nargs="+")
    ap.add_argument("--out", default=os.path.join(ROOT, "profiles", "pmc_traffic.json"))
    a = ap.parse_args()
    try:
        with open(a.out) as f:
            merged = json.load(f)
    except (OSError, ValueError):
        merged = {}
    for p in a.summaries:
        with open(p) as f:
            part = json.load(f)
        for k, v in part.items():
            if not isinstance(v, dict) or "lib_sha256" not in v or "hbm_bytes_per_launch" not in v:
                raise SystemExit(f"{p}: entry {k} is not a stamped PMC record")
            merged[k] = v
    with open(a.out, "w") as f:
        json.dump(merged, f, indent=1)
    print(json.dumps({k: [v["hbm_bytes_per_launch"], v["lib_sha256"][:12]] for k, v in merged.items()}))


if __name__ == "__main__":
    main()
