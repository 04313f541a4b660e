"""Reference-dot mode names the host it reproduces (Next 5).

EDT_RL/crossover.py:27-40 forms the SLERP coefficients with numpy float32 arccos / sin, whose bits
depend on the SIMD loop numpy dispatches to at run time (AVX512_SKX's SVML arccos vs the baseline
libm one, AVX512_SKX / AVX2 / baseline sin), and the dot with numpy's BLAS sdot. ops.RefDot records
the modelled host (dot kernel + the float32 loop targets); tests/golden/refdot_host.json is the
host the golden SLERP outputs were recorded on (tests/golden/gen_refdot_host.py). Pinned here:
  * RefDot's defaults are that record;
  * on a host that matches it the mode stays silent and the golden outputs reproduce bit for bit
    from the recorded dots (test_refdot_reach_cpu.py); on one that does not it warns;
  * on this same machine with numpy's AVX-512 loops switched off (NPY_DISABLE_CPU_FEATURES, a
    subprocess) the dispatch differs, numpy's own coefficients no longer reproduce the golden
    outputs, and RefDot warns — or raises with strict=True — instead of going on silently."""
import json
import os
import subprocess
import sys
import warnings

import pytest

from evolutionarydistributedtraining_amd import ops

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
RECORD = json.load(open(os.path.join(ROOT, "tests", "golden", "refdot_host.json")))


def test_refdot_defaults_are_the_golden_host():
    r = ops.RefDot()
    assert dict(r.coef_dispatch) == RECORD["coef_dispatch"]
    assert r.dot_kernel == RECORD["blas"]
    d = r.describe()
    assert d["coef_dispatch"] == RECORD["coef_dispatch"] and d["dot_kernel"] == RECORD["blas"]
    assert set(d["host"]["coef_dispatch"]) == {"arccos", "sin"}


def test_this_host_against_the_record():
    host = ops.host_dispatch()
    r = ops.RefDot(coef_dispatch=tuple((k, v) for k, v in sorted(RECORD["coef_dispatch"].items())))
    ops._REFDOT_CHECKED.clear()
    if host["coef_dispatch"] == RECORD["coef_dispatch"] and host["blas"] == RECORD["blas"]:
        assert r.host_mismatch() == []
        with warnings.catch_warnings():
            warnings.simplefilter("error")
            r.check_host()
    else:
        assert r.host_mismatch()
        with pytest.warns(ops.RefDotHostWarning):
            r.check_host()


def test_a_modelled_host_that_differs_warns_once_or_raises():
    ops._REFDOT_CHECKED.clear()
    other = ops.RefDot(coef_dispatch=(("arccos", "baseline(SSE SSE2 SSE3)"), ("sin", "AVX2")))
    assert len(other.host_mismatch()) >= 1 or ops.host_dispatch()["coef_dispatch"]["sin"] == "AVX2"
    if other.host_mismatch():
        with pytest.warns(ops.RefDotHostWarning, match="arccos|sin"):
            other.check_host()
        with warnings.catch_warnings():
            warnings.simplefilter("error")
            other.check_host()                      # once per setting
        with pytest.raises(ops.L.EdtError, match="not the one it reproduces"):
            ops.RefDot(coef_dispatch=other.coef_dispatch, strict=True).check_host()
    wrong_blas = ops.RefDot(dot_kernel="openblas 0.3.29 Haswell")
    if ops.host_dispatch()["blas"] is not None:
        assert any("BLAS" in m for m in wrong_blas.host_mismatch())


_CHILD = r'''
import json, sys, warnings
import numpy as np
sys.path.insert(0, sys.argv[1])
from evolutionarydistributedtraining_amd import ops
from tests.golden_data import Golden
g = Golden()
tens = g.tensors("slerp")
bad = 0
for c in g.slerp_cases():
    v0 = tens[f"{c['inputs']}/v0"].float().numpy().ravel()
    v1 = tens[f"{c['inputs']}/v1"].float().numpy().ravel()
    c0, c1 = ops.reference_coefficients(np.float32([c["ref_dot"]]), np.float64([c["t"]]))[0]
    want = tens[f"{c['name']}/out"].float().numpy().ravel()
    bad += int(not np.array_equal((c0 * v0 + c1 * v1).view(np.int32), want.view(np.int32)))
with warnings.catch_warnings(record=True) as w:
    warnings.simplefilter("always")
    ops.RefDot().check_host()
try:
    ops.RefDot(strict=True).check_host()
    raised = False
except ops.L.EdtError:
    raised = True
print(json.dumps({"host": ops.host_dispatch(), "golden_mismatch": bad,
                  "warned": any(issubclass(x.category, ops.RefDotHostWarning) for x in w), "raised": raised}))
'''


def test_another_dispatch_breaks_the_golden_bits_and_is_flagged():
    if ops.host_dispatch()["coef_dispatch"] != RECORD["coef_dispatch"]:
        pytest.skip("this host is not the recorded one (covered by test_this_host_against_the_record)")
    env = dict(os.environ, NPY_DISABLE_CPU_FEATURES="AVX512F AVX512CD AVX512_SKX AVX512_CLX AVX512_CNL "
                                                    "AVX512_ICL AVX512_SPR")
    out = subprocess.run([sys.executable, "-c", _CHILD, ROOT], env=env, capture_output=True, text=True,
                         timeout=300, cwd=ROOT)
    assert out.returncode == 0, out.stderr[-2000:]
    res = json.loads(out.stdout.strip().splitlines()[-1])
    assert res["host"]["coef_dispatch"] != RECORD["coef_dispatch"], res
    assert res["golden_mismatch"] > 0, res          # the dispatch changes the reference's bits
    assert res["warned"] and res["raised"], res


def test_host_dispatch_without_numpy_introspect(monkeypatch):
    """numpy < 2 has no numpy.lib.introspect. The dispatch is then recorded as unknown
    (no ImportError on every reference-dot merge), which host_mismatch reports — a warning, or
    EdtError with strict=True."""
    import sys

    import numpy.lib
    import pytest

    from evolutionarydistributedtraining_amd import _lib as L
    from evolutionarydistributedtraining_amd import ops
    monkeypatch.setattr(ops, "_HOST_DISPATCH", None)
    monkeypatch.delattr(numpy.lib, "introspect", raising=False)
    monkeypatch.setitem(sys.modules, "numpy.lib.introspect", None)
    host = ops.host_dispatch()
    assert host["coef_dispatch"] == {"arccos": "unknown", "sin": "unknown"}
    bad = ops.RefDot().host_mismatch()
    assert any("unknown" in b for b in bad)
    monkeypatch.setattr(ops, "_REFDOT_CHECKED", set())
    with pytest.raises(L.EdtError):
        ops.RefDot(strict=True).check_host()
    monkeypatch.setattr(ops, "_HOST_DISPATCH", None)
