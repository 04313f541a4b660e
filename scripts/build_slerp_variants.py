"""Build-time variants of the chunk-sum passes (edt_slerp.hip) into variants_slerp/,
for scripts/slerp_spec_probe.py --variants variants_slerp (timed beside the in-tree library).

    python scripts/build_slerp_variants.py [name ...]
"""
import os
import sys
from concurrent.futures import ThreadPoolExecutor

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
OUT = os.path.join(ROOT, "variants_slerp")

VARIANTS = {
    "tpw4": ["-DEDT_SLERP_STATS_TPW=4"],
    "tpw8": ["-DEDT_SLERP_STATS_TPW=8"],
    "nont": ["-DEDT_NT_SLERP=0"],
    "waverows": ["-DEDT_SLERP_SPEC_WG_ROWS=0"],
    "gramprefetch": ["-DEDT_GRAM_PREFETCH=1"],
    "gramnt": ["-DEDT_GRAM_NT=1"],
    "gramntpf": ["-DEDT_GRAM_NT=1", "-DEDT_GRAM_PREFETCH=1"],
    "gramregs3": ["-DEDT_GRAM_PREFETCH=0"],
    "grampf3": ["-DEDT_GRAM_MIN_BLOCKS=3"],
    "gramnont": ["-DEDT_GRAM_NT=0"],
}


def main():
    from evolutionarydistributedtraining_amd.build import build_library
    names = sys.argv[1:] or list(VARIANTS)
    os.makedirs(OUT, exist_ok=True)
    for f in os.listdir(OUT):
        if f.endswith(".so") and f[3:-3] not in names:
            os.remove(os.path.join(OUT, f))
    with ThreadPoolExecutor(3) as ex:
        list(ex.map(lambda n: build_library(force=True, extra_flags=VARIANTS[n], out=os.path.join(OUT, f"lib{n}.so")),
                    names))
    print("built", names)


if __name__ == "__main__":
    main()
