"""How much numpy's float32 arccos / sin depend on the SIMD loop they dispatch to (the reason
ops.RefDot records and checks the dispatch): the same 400k float32 dots (200k uniform in [-1, 1],
200k within 1e-4 of DOT_THRESHOLD) through arccos and sin(th * t) under this process's dispatch and
in child processes with numpy's AVX-512 (then also AVX2 / FMA3 / AVX) loops disabled
(NPY_DISABLE_CPU_FEATURES); prints the dispatch targets and the count of differing results.

    python scripts/numpy_dispatch_probe.py
"""
import json
import os
import subprocess
import sys

CHILD = r'''
import json, sys
import numpy as np
from numpy.lib import introspect
rng = np.random.default_rng(0)
d = np.concatenate([rng.uniform(-1, 1, 200000), 0.9995 + rng.uniform(-1e-4, 1e-4, 200000)]).astype(np.float32)
th0 = np.arccos(d)
s = np.sin(th0 * np.float32(0.43))
disp = {f: introspect.opt_func_info(func_name=f"^{f}$", signature="float32")[f]["ff"]["current"] for f in ("arccos", "sin")}
np.save(sys.argv[1], np.stack([th0, s]))
print(json.dumps(disp))
'''
AVX512 = "AVX512F AVX512CD AVX512_SKX AVX512_CLX AVX512_CNL AVX512_ICL AVX512_SPR"


def main():
    import tempfile

    import numpy as np
    runs = {"this_host": None, "no_avx512": AVX512, "baseline_only": AVX512 + " AVX2 FMA3 F16C AVX"}
    out, arrs = {}, {}
    with tempfile.TemporaryDirectory() as tmp:
        for name, off in runs.items():
            env = dict(os.environ)
            if off:
                env["NPY_DISABLE_CPU_FEATURES"] = off
            path = os.path.join(tmp, name + ".npy")
            p = subprocess.run([sys.executable, "-c", CHILD, path], env=env, capture_output=True, text=True, timeout=120)
            if p.returncode:
                raise SystemExit(p.stderr)
            out[name] = {"dispatch": json.loads(p.stdout.strip().splitlines()[-1])}
            arrs[name] = np.load(path)
    for name in runs:
        a, b = arrs["this_host"], arrs[name]
        out[name]["arccos_differs"] = int((a[0].view(np.int32) != b[0].view(np.int32)).sum())
        out[name]["sin_differs"] = int((a[1].view(np.int32) != b[1].view(np.int32)).sum())
    print(json.dumps({"probe": "numpy_dispatch", "values": 400000, "runs": out}))


if __name__ == "__main__":
    main()
