"""Reference-dot mode on the MI355X (ops.RefDot -> edt_slerp_refdot_flags / edt_slerp_refdot /
edt_slerp_refdot_coef): the device recomputes the reference's own fp32 dot of EDT_RL/crossover.py:20-29
(BLAS sdot norms + numpy's buffered pairwise sum of the normalised products) bit for bit.

  * the dot of every golden SLERP case equals the reference's recorded dot, bit for bit, and the
    restatement's (oracle.ref_slerp_dot) — fp32 and bf16 inputs, one multi-segment launch;
  * random layouts whose sizes cross every block edge of both reductions, BLAS thread splits 1 / 3;
  * the 24 DOT_THRESHOLD cases (tests/golden/slerp_threshold.json): in this mode the kernel takes
    the reference's branch on every case, the four straddles included, and its output is within
    the ordinary 2e-6 SLERP bar of the reference's (the lerp branch bit for bit) — the fp64 default
    keeps its documented contract (tests/test_slerp_threshold.py);
  * band flags: only segments near the threshold are recomputed, the others keep the fp64 dot."""
import json
import os

import numpy as np
import pytest
import torch
from safetensors.torch import load_file

from tests.golden.threshold_inputs import digest, make_pair, sample_index

pytestmark = pytest.mark.gpu
GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
THR = 0.9995


@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.skip("needs a HIP device")
    return torch.device("cuda:0")


def _ref_dots(dev, parts, threads=1, band=-1.0, t=0.5):
    """One arena of the given (v0, v1) segments; returns (device dots after the ref pass, plan)."""
    from evolutionarydistributedtraining_amd import ops
    offs = [0]
    for a, _ in parts:
        offs.append(offs[-1] + a.numel())
    dt = parts[0][0].dtype
    v0 = torch.cat([a.reshape(-1) for a, _ in parts]).to(dev, dt)
    v1 = torch.cat([b.reshape(-1) for _, b in parts]).to(dev, dt)
    plan = ops.make_slerp_plan(offs, dev)
    out = torch.empty(offs[-1], dtype=torch.float32, device=dev)
    tt = torch.full((len(parts),), t, dtype=torch.float64, device=dev)
    ops.slerp_arena(plan, v0, v1, out, tt, ref_dot=ops.RefDot(threads=threads, band=band))
    torch.cuda.synchronize()
    return plan.dots[:len(parts)].cpu(), plan, out.cpu()


@pytest.mark.parametrize("in_dtype", ["f32", "bf16"])
def test_refdot_golden_cases(oracle, golden, dev, in_dtype):
    tens = golden.tensors("slerp")
    cases, seen = [], set()
    for c in golden.slerp_cases():
        if c["in_dtype"] == in_dtype and c["inputs"] not in seen:
            seen.add(c["inputs"])
            cases.append(c)
    parts = [(tens[f"{c['inputs']}/v0"].contiguous(), tens[f"{c['inputs']}/v1"].contiguous()) for c in cases]
    dots, _, _ = _ref_dots(dev, parts)
    for c, (a, b), d in zip(cases, parts, dots.tolist()):
        want, _, _ = oracle.ref_slerp_dot(a, b)
        assert np.float32(d) == want, c["name"]
        assert d == c["ref_dot"], c["name"]


@pytest.mark.parametrize("threads", [1, 3])
@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
def test_refdot_random_layouts(oracle, dev, threads, dt):
    g = torch.Generator().manual_seed(17 + threads)
    sizes = [1, 7, 31, 32, 33, 63, 64, 65, 127, 128, 129, 8191, 8192, 8193, 16385, 65536, 65537, 131073, 300001]
    parts = []
    for i, n in enumerate(sizes):
        x = torch.randn(n, generator=g) * (0.02 if i % 2 else 1.5)
        y = x + torch.randn(n, generator=g) * 0.02 * (0.01 if i % 3 else 0.5)
        parts.append((x.to(dt), y.to(dt)))
    parts.append((torch.zeros(5, dtype=dt), torch.ones(5, dtype=dt)))        # a zero norm: no division
    dots, _, _ = _ref_dots(dev, parts, threads=threads)
    for (a, b), d in zip(parts, dots.tolist()):
        want, _, _ = oracle.ref_slerp_dot(a, b, threads=threads)
        assert np.float32(d) == want, (a.numel(), d, float(want))


def _threshold_fixture():
    with open(os.path.join(GOLDEN, "slerp_threshold.json")) as f:
        meta = json.load(f)
    return meta["cases"], load_file(os.path.join(GOLDEN, "slerp_threshold.safetensors"))


THR_CASES, _ = _threshold_fixture()


@pytest.mark.parametrize("band", [-1.0, 1e-4])
@pytest.mark.parametrize("c", THR_CASES, ids=[c["name"] for c in THR_CASES])
def test_refdot_mode_takes_the_reference_branch_at_threshold(dev, c, band):
    from evolutionarydistributedtraining_amd import ops
    _, tensors = _threshold_fixture()
    if f"{c['name']}/v0" in tensors:
        a, b = tensors[f"{c['name']}/v0"], tensors[f"{c['name']}/v1"]
    else:
        a, b = make_pair(c["seed"], c["n"], c["dtype"], c["noise_scale"])
    assert digest(a, b) == c["sha256"]
    n = c["n"]
    idx = sample_index(n)
    plan = ops.make_slerp_plan([0, n], dev)
    for o in c["outputs"]:
        t = torch.tensor([o["t"]], dtype=torch.float64, device=dev)
        out = torch.empty(n, dtype=torch.float32, device=dev)
        ops.slerp_arena(plan, a.to(dev), b.to(dev), out, t, ref_dot=ops.RefDot(band=band))
        dot = plan.dots[0].item()
        assert dot == c["ref_dot"], (c["name"], dot, c["ref_dot"])        # the reference's own dot
        got, ref = out.cpu()[idx], tensors[f"{o['key']}/out"]
        if c["ref_lerp_branch"]:
            assert torch.equal(got.view(torch.int32), ref.view(torch.int32)), c["name"]
        else:
            v0, v1 = a.double()[idx], b.double()[idx]
            th = np.arccos(np.float32(dot), dtype=np.float32)
            c0 = float(np.sin(th - th * np.float32(o["t"])) / np.sin(th))
            c1 = float(np.sin(th * np.float32(o["t"])) / np.sin(th))
            bar = 2e-6 * (abs(c0) * v0.abs() + abs(c1) * v1.abs())
            assert ((got.double() - ref.double()).abs() <= bar + 1e-30).all(), c["name"]


def test_refdot_band_flags_only_near_threshold(oracle, dev):
    """band > 0: a far segment keeps the fp64 dot (not recomputed), a near one gets the reference's."""
    c = next(c for c in THR_CASES if c["ref_lerp_branch"] != c["exact_lerp_branch"])     # a straddle
    _, tensors = _threshold_fixture()
    if f"{c['name']}/v0" in tensors:
        a, b = tensors[f"{c['name']}/v0"], tensors[f"{c['name']}/v1"]
    else:
        a, b = make_pair(c["seed"], c["n"], c["dtype"], c["noise_scale"])
    g = torch.Generator().manual_seed(23)
    far = (torch.randn(70001, generator=g).to(a.dtype), torch.randn(70001, generator=g).to(a.dtype))   # dot ~ 0
    parts = [far, (a, b)]
    dots_band, plan, _ = _ref_dots(dev, parts, band=1e-3)
    assert plan._refdot_flag[:2].cpu().tolist() == [0, 1]
    assert dots_band[1].item() == c["ref_dot"]
    dots_all, _, _ = _ref_dots(dev, parts, band=-1.0)
    want_far, _, _ = oracle.ref_slerp_dot(*far)
    assert np.float32(dots_all[0].item()) == want_far
    assert abs(dots_band[0].item() - float(want_far)) < 1e-5                # the fp64 dot, the usual bar


def test_refdot_large_tensor(oracle, dev):
    """One 67.9M-element tensor (a Qwen2.5-7B MLP weight, 18944 x 3584), bf16, every segment mode:
    the device dot equals the restatement's; records the time of the reference-dot passes."""
    import time
    g = torch.Generator(device=dev).manual_seed(29)
    n = 18944 * 3584
    x = (torch.randn(n, device=dev, generator=g) * 0.02)
    y = (x + torch.randn(n, device=dev, generator=g) * 0.02 * 0.02).bfloat16()
    x = x.bfloat16()
    from evolutionarydistributedtraining_amd import ops
    plan = ops.make_slerp_plan([0, n], dev)
    out = torch.empty(n, dtype=torch.bfloat16, device=dev)
    t = torch.tensor([0.5], dtype=torch.float64, device=dev)
    ops.slerp_arena(plan, x, y, out, t, ref_dot=ops.RefDot())
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    ops.slerp_arena(plan, x, y, out, t, ref_dot=ops.RefDot())
    torch.cuda.synchronize()
    ms = 1e3 * (time.perf_counter() - t0)
    want, _, _ = oracle.ref_slerp_dot(x.cpu(), y.cpu())
    assert np.float32(plan.dots[0].item()) == want
    d = os.environ.get("EDT_RECORD_DIR")
    if d:
        os.makedirs(d, exist_ok=True)
        with open(os.path.join(d, "refdot_large.json"), "w") as f:
            json.dump({"elements": n, "dtype": "bf16", "merge_with_refdot_ms": round(ms, 3)}, f)
