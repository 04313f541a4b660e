"""Records the host side of the reference-dot mode on the machine that generated tests/golden/
(gen_golden.py, gen_slerp_threshold.py ran on this image: numpy 2.2.6 with its bundled OpenBLAS
0.3.29): which SIMD targets numpy's float32 arccos / sin dispatch to and numpy's BLAS core. The
golden SLERP outputs are the reference's bits under exactly this dispatch; ops.RefDot's defaults
are this record (tests/test_refdot_host_cpu.py pins both). No reference code is imported.

    python tests/golden/gen_refdot_host.py   # writes tests/golden/refdot_host.json
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def main():
    from evolutionarydistributedtraining_amd.ops import host_dispatch
    rec = dict(host_dispatch())
    rec["note"] = ("host of the golden SLERP fixtures: numpy float32 arccos / sin SIMD targets "
                   "(numpy.lib.introspect.opt_func_info) and numpy's BLAS (threadpoolctl)")
    out = os.path.join(os.path.dirname(os.path.abspath(__file__)), "refdot_host.json")
    with open(out, "w") as f:
        json.dump(rec, f, indent=1)
    print(json.dumps(rec))


if __name__ == "__main__":
    main()
