"""Pin the CPU oracle against the golden vectors produced by the reference's own code.

These run on CPU (no GPU): they are what makes the oracle trustworthy as the checker of the HIP
kernels. Bar: bit-exact on every case (DiLoCo outer step, EDT pair merge, lerp, SLERP).
"""
import json
import os

import pytest
import torch

from tests.golden_data import GOLDEN_DIR, bits, flat

with open(os.path.join(GOLDEN_DIR, "manifest.json")) as _f:
    _MANIFEST = json.load(_f)
N_DILOCO = len(_MANIFEST["diloco"])
N_PAIR = len(_MANIFEST["pair_merge"])


def _momentum_for(case_step, mu, gdt, n, prev_buf):
    if mu == 0:
        return None, False
    if prev_buf is None:
        return torch.zeros(n, dtype=gdt), False
    return prev_buf.clone(), True


@pytest.mark.parametrize("idx", range(N_DILOCO))
def test_diloco_oracle_bit_exact(golden, oracle, idx):
    c = golden.diloco_cases()[idx]
    T = len(c["shapes"])
    prev_buf = None
    for step in c["steps"]:
        pre = step["prefix"]
        theta = flat(golden.tlist("diloco", f"{pre}/base", T)).contiguous()
        workers = [flat(golden.tlist("diloco", f"{pre}/worker{k}", T)).contiguous() for k in range(c["K"])]
        mom, has = _momentum_for(step, c["momentum"], theta.dtype, theta.numel(), prev_buf)
        tail = oracle.torch_cpu_tail_mask([int(torch.Size(s).numel()) for s in c["shapes"]])
        oracle.outer_step(theta, workers, mom, has, c["lr"], c["momentum"], c["nesterov"], tail)
        want = flat(golden.tlist("diloco", f"{pre}/out_theta", T))
        assert theta.dtype == want.dtype
        assert torch.equal(bits(theta), bits(want)), f"{pre}: theta mismatch"
        if step["has_out_buf"]:
            want_b = flat(golden.tlist("diloco", f"{pre}/out_buf", T))
            assert torch.equal(bits(mom), bits(want_b)), f"{pre}: momentum mismatch"
            prev_buf = mom
        else:
            assert mom is None


def test_golden_case_counts(golden):
    assert N_DILOCO == 30 and N_PAIR == 8
    ks = {c["K"] for c in golden.diloco_cases()}
    assert ks == {1, 2, 3, 8}


def pair_inputs(golden, c):
    """Inputs of one pair-merge case, with the reference's parent-optimizer rules applied
    (EDT_LM/train/crossover.py:187-227): both -> parent 1's state; one -> that one."""
    pre, T = c["name"], c["n_tensors"]
    g = lambda tag: flat(golden.tlist("pair_merge", f"{pre}/{tag}", T)).contiguous()
    b1, b2, m1, m2 = g("b1"), g("b2"), g("m1"), g("m2")
    bdt = torch.float32 if c["base_dtype"] == "f32" else torch.bfloat16
    lr, mu, nest = c["call_lr"], c["call_momentum"], c["call_nesterov"]
    mom, has = None, False
    if c["parent1_optim"] or c["parent2_optim"]:
        mom = (g("buf1") if c["parent1_optim"] else g("buf2")).to(bdt)
        has = True
        grp = c["saved_param_group"]          # load_state_dict replaces the group's settings
        lr, mu, nest = grp["lr"], grp["momentum"], grp["nesterov"]
    if mu != 0 and mom is None:
        mom = torch.zeros(b1.numel(), dtype=bdt)
    if mu == 0:
        mom, has = None, False
    return dict(b1=b1, b2=b2, m1=m1, m2=m2, bdt=bdt, lr=lr, mu=mu, nesterov=nest, mom=mom, has=has,
                want_base=g("merged_base"), want_theta=g("out_theta"),
                want_buf=g("out_buf") if c["has_out_buf"] else None)


@pytest.mark.parametrize("idx", range(N_PAIR))
def test_pair_merge_oracle_bit_exact(golden, oracle, idx):
    c = golden.pair_cases()[idx]
    p = pair_inputs(golden, c)
    base = oracle.lerp(0.5, p["b1"], p["b2"]).to(p["bdt"])
    assert torch.equal(bits(base), bits(p["want_base"])), "run_linear_merge_5050 mismatch"
    out = torch.empty(p["b1"].numel(), dtype=p["bdt"])
    tail = oracle.torch_cpu_tail_mask([int(torch.Size(s).numel()) for s in c["shapes"]])
    oracle.pair_merge(p["b1"], p["b2"], p["m1"], p["m2"], out, p["mom"], p["has"], p["lr"], p["mu"],
                      p["nesterov"], tail)
    assert torch.equal(bits(out), bits(p["want_theta"])), f"{c['name']}: theta mismatch"
    if p["want_buf"] is not None:
        assert torch.equal(bits(p["mom"]), bits(p["want_buf"].to(p["bdt"]))), "momentum mismatch"
    # the base-given form (run_sgd on an existing base model) agrees too
    out2 = torch.empty_like(out)
    mom2 = pair_inputs(golden, c)["mom"]      # fresh copy: p["mom"] was updated in place
    oracle.pair_merge(base, None, p["m1"], p["m2"], out2, mom2, p["has"], p["lr"], p["mu"], p["nesterov"],
                      tail)
    assert torch.equal(bits(out2), bits(out))


def test_slerp_oracle_bit_exact(golden, oracle):
    t = golden.tensors("slerp")
    n_lerp = 0
    for c in golden.slerp_cases():
        v0, v1 = t[f"{c['inputs']}/v0"], t[f"{c['inputs']}/v1"]
        res, dot, lerp_branch = oracle.slerp_parts(c["t"], v0, v1)
        want = t[f"{c['name']}/out"]
        assert lerp_branch == c["lerp_branch"], c["name"]
        assert float(dot) == c["ref_dot"], c["name"]
        got = torch.from_numpy(res)
        assert got.shape == want.shape and got.dtype == want.dtype
        assert torch.equal(bits(got), bits(want)), c["name"]
        n_lerp += lerp_branch
    assert 0 < n_lerp < len(golden.slerp_cases())


def test_diloco_large_bf16_parallel_tails(golden, oracle):
    """A bf16 case with tensors above torch's parallel grain: the reference's scalar tails fall at
    the end of every parallel chunk; the oracle's tail model reproduces it bit for bit."""
    c = golden.manifest["diloco_large"]
    T = len(c["shapes"])
    numels = [int(torch.Size(s).numel()) for s in c["shapes"]]
    tail = oracle.torch_cpu_tail_mask(numels, num_threads=c["torch_num_threads"])
    pre = c["name"]
    theta = flat(golden.tlist("diloco", f"{pre}/s0/base", T)).contiguous()
    mom = torch.zeros_like(theta)
    for step in (0, 1):
        ws = [flat(golden.tlist("diloco", f"{pre}/s{step}/worker{k}", T)).contiguous() for k in range(c["K"])]
        oracle.outer_step(theta, ws, mom, step == 1, c["lr"], c["momentum"], c["nesterov"], tail)
        want = flat(golden.tlist("diloco", f"{pre}/s{step}/out_theta", T))
        assert torch.equal(bits(theta), bits(want)), step
    assert torch.equal(bits(mom), bits(flat(golden.tlist("diloco", f"{pre}/s1/out_buf", T))))
    # and without the tail model the differences are confined to those tail elements
    assert int(tail.sum()) < 0.01 * tail.numel()


def test_torch_loop_restatement_matches_c_oracle(oracle):
    """oracle.torch_loop_outer_step (the reference's loop as bench.py times it on the host) computes
    what the C oracle does, bit for bit, over two generations with the carried SGD buffer (fp32)."""
    g = torch.Generator().manual_seed(4)
    shapes = [(33, 7), (5,), (300,), (64, 64)]
    K = 3
    base = [torch.randn(s, generator=g) * 0.02 for s in shapes]
    workers = [[p + torch.randn(p.shape, generator=g) * 1e-3 for p in base] for _ in range(K)]
    flat = torch.cat([p.reshape(-1) for p in base])
    wflat = [torch.cat([p.reshape(-1) for p in w]) for w in workers]
    mom = torch.zeros_like(flat)
    opt = None
    for gen in range(2):
        opt = oracle.torch_loop_outer_step(base, workers, opt, 0.7, 0.9, True)
        oracle.outer_step(flat, wflat, mom, gen > 0, 0.7, 0.9, True)
        got = torch.cat([p.detach().reshape(-1) for p in base])
        assert torch.equal(got.view(torch.int32), flat.view(torch.int32)), gen
