"""Generate the golden vectors for the outer-loop sync hot path FROM THE REFERENCE ITSELF.

Test infrastructure only. This script runs in the build container (it needs `/root/reference`
and `transformers`); it is never imported by the tests, `smoke()` or `bench.py`, and nothing
of the reference is copied: the reference's own functions are imported by path (or, for the
DiLoCo block that lives at module level, compiled from the source text and exec'd against stub
models) and only their numeric inputs/outputs are written out.

Reference code exercised (paths relative to /root/reference):
  EDT_LM/diloco.py:238-289            DiLoCo outer step block (defaults lr .7, mu .9, nesterov)
  EDT_LM/diloco_sim.py:233-299        same block with the sim defaults (lr 1.0, mu 0, plain)
  EDT_LM/train/crossover.py:150-237   run_linear_merge_5050 + run_sgd (EDT pair merge)
  EDT_LM/train/crossover.py:318-321   uniform_dna_crossover
  EDT_RL/crossover.py:11-201          slerp / interpolate_t / run_slerp_merge / crossover
  EDT_EVOMERGE/train/crossover.py:14-146  slerp + run_slerp_merge_from_config (bf16 models)

Output: tests/golden/{diloco,pair_merge,slerp,merge_models}.safetensors + manifest.json

    python tests/golden/gen_golden.py
"""
from __future__ import annotations

import copy
import importlib.util
import json
import os
import tempfile
import textwrap

import numpy as np
import torch
from safetensors.torch import load_file, save_file

REF = "/root/reference"
HERE = os.path.dirname(os.path.abspath(__file__))

DILOCO_BLOCKS = {
    # name: (file, first line, last line, block defaults (lr, mu, nesterov))
    "diloco": ("EDT_LM/diloco.py", 238, 289, (0.7, 0.9, True)),
    "diloco_sim": ("EDT_LM/diloco_sim.py", 233, 299, (1.0, 0.0, False)),
}

SHAPES = [(1,), (7,), (33, 5), (16, 16), (3, 17, 3), (64,)]
DTYPES = {"f32": torch.float32, "bf16": torch.bfloat16}


def _load_module(name: str, rel: str):
    spec = importlib.util.spec_from_file_location(name, os.path.join(REF, rel))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def _block(rel: str, first: int, last: int):
    with open(os.path.join(REF, rel)) as f:
        lines = f.read().splitlines()[first - 1:last]
    return compile(textwrap.dedent("\n".join(lines)), f"{rel}:{first}-{last}", "exec")


class StubModel:
    """Stands in for an HF model: the DiLoCo block only calls `.parameters()`."""

    def __init__(self, tensors):
        self._params = [torch.nn.Parameter(t.clone()) for t in tensors]

    def parameters(self):
        return iter(self._params)


def _base_tensors(gen: torch.Generator, dtype) -> list[torch.Tensor]:
    out = []
    for s in SHAPES:
        t = torch.randn(s, generator=gen) * 0.02
        out.append(t)
    # edge values in the small tensors: zeros of both signs, an exact-1 norm weight, a large value
    out[0].view(-1)[0] = 0.0
    e = out[1].view(-1)
    e[0], e[1], e[2], e[3] = -0.0, 1.0, 3.0, 1e-30
    return [t.to(dtype) for t in out]


def _worker_tensors(gen, base: list[torch.Tensor], dtype, k: int) -> list[torch.Tensor]:
    out = []
    for i, b in enumerate(base):
        w = b.float() + torch.randn(b.shape, generator=gen) * 1e-3
        if i == 1:
            flat = w.view(-1)
            flat[4] = b.view(-1)[4].float()          # zero delta
            flat[5] = b.view(-1)[5].float() + 0.25 * (k + 1)   # large delta
        out.append(w.to(dtype))
    return out


def _exec_diloco(code, base, workers, evo, prev_opt):
    ns = dict(
        torch=torch, optim=torch.optim,
        base_model=StubModel(base),
        trained_models=[StubModel(w) for w in workers],
        num_models=len(workers), EVOLUTION=evo, outer_optimizer=prev_opt,
    )
    exec(code, ns)
    params = list(ns["base_model"].parameters())
    opt = ns["outer_optimizer"]
    theta = [p.detach().clone() for p in params]
    # clone: the next generation's load_state_dict reuses these buffers and mutates them in place
    bufs = [opt.state[p]["momentum_buffer"].clone()
            if p in opt.state and opt.state[p].get("momentum_buffer") is not None else None
            for p in params]
    return theta, bufs, opt


def gen_diloco(manifest, tensors):
    seed = 1000
    cases = []
    variants = [
        ("diloco", {}, [1, 2, 3, 8]),
        ("diloco_sim", {}, [1, 2, 3, 8]),
        ("diloco", {"OUTER_NESTEROV": False}, [3]),
        ("diloco", {"OUTER_LR": 0.5, "OUTER_MOMENTUM": 0.8}, [2]),
    ]
    regimes = [("f32", "f32"), ("bf16", "bf16"), ("f32", "bf16")]   # (global dtype, worker dtype)
    for block_name, evo, ks in variants:
        rel, first, last, (lr0, mu0, nest0) = DILOCO_BLOCKS[block_name]
        code = _block(rel, first, last)
        lr = evo.get("OUTER_LR", lr0)
        mu = evo.get("OUTER_MOMENTUM", mu0)
        nest = evo.get("OUTER_NESTEROV", nest0)
        for gdt, wdt in regimes:
            for K in ks:
                seed += 1
                gen = torch.Generator().manual_seed(seed)
                name = f"diloco/{block_name}_lr{lr}_mu{mu}_n{int(nest)}_{gdt}_{wdt}_K{K}"
                base = _base_tensors(gen, DTYPES[gdt])
                opt = None
                steps = []
                for step in range(2):
                    workers = [_worker_tensors(gen, base, DTYPES[wdt], k) for k in range(K)]
                    theta, bufs, opt = _exec_diloco(code, base, workers, dict(evo), opt)
                    pre = f"{name}/s{step}"
                    for i, t in enumerate(base):
                        tensors[f"{pre}/base/{i}"] = t
                    for k, w in enumerate(workers):
                        for i, t in enumerate(w):
                            tensors[f"{pre}/worker{k}/{i}"] = t
                    for i, t in enumerate(theta):
                        tensors[f"{pre}/out_theta/{i}"] = t
                    has_buf = bufs[0] is not None
                    if has_buf:
                        for i, t in enumerate(bufs):
                            tensors[f"{pre}/out_buf/{i}"] = t
                    steps.append({"prefix": pre, "has_out_buf": has_buf})
                    base = theta
                cases.append({
                    "name": name, "source": f"{rel}:{first}-{last}", "K": K,
                    "global_dtype": gdt, "worker_dtype": wdt, "lr": lr, "momentum": mu,
                    "nesterov": nest, "shapes": [list(s) for s in SHAPES], "steps": steps,
                })
    manifest["diloco"] = cases
    # one large bf16 case: tensors above torch's 32768-element grain are split over threads, and
    # every parallel chunk has its own scalar tail (pins the oracle's tail model at scale)
    rel, first, last, (lr, mu, nest) = DILOCO_BLOCKS["diloco"]
    code = _block(rel, first, last)
    gen = torch.Generator().manual_seed(4321)
    shapes = [(70_001,), (257, 160)]
    base = [(torch.randn(sh, generator=gen) * 0.02).bfloat16() for sh in shapes]
    workers = [[(b.float() + torch.randn(b.shape, generator=gen) * 1e-3).bfloat16() for b in base] for _ in range(3)]
    opt = None
    theta0, _, opt = _exec_diloco(code, base, workers, {}, opt)
    workers2 = [[(b.float() + torch.randn(b.shape, generator=gen) * 1e-3).bfloat16() for b in theta0] for _ in range(3)]
    theta1, bufs1, _ = _exec_diloco(code, theta0, workers2, {}, opt)
    pre = "diloco_large"
    for i, t in enumerate(base):
        tensors[f"{pre}/s0/base/{i}"] = t
    for k in range(3):
        for i in range(len(shapes)):
            tensors[f"{pre}/s0/worker{k}/{i}"] = workers[k][i]
            tensors[f"{pre}/s1/worker{k}/{i}"] = workers2[k][i]
    for i in range(len(shapes)):
        tensors[f"{pre}/s0/out_theta/{i}"] = theta0[i]
        tensors[f"{pre}/s1/out_theta/{i}"] = theta1[i]
        tensors[f"{pre}/s1/out_buf/{i}"] = bufs1[i]
    manifest["diloco_large"] = {"name": pre, "source": f"{rel}:{first}-{last}", "K": 3, "dtype": "bf16",
                                "lr": lr, "momentum": mu, "nesterov": nest, "shapes": [list(x) for x in shapes],
                                "torch_num_threads": torch.get_num_threads()}


# ----------------------------------------------------------------------------------------
# EDT pair merge (EDT_LM/train/crossover.py:150-237)

def _tiny_llama_config(dtype: str):
    from transformers import LlamaConfig
    return LlamaConfig(vocab_size=24, hidden_size=8, intermediate_size=16, num_hidden_layers=4,
                       num_attention_heads=2, num_key_value_heads=1, tie_word_embeddings=False,
                       dtype=dtype)


def _llama_with(cfg, tensors, dtype):
    from transformers import LlamaForCausalLM
    m = LlamaForCausalLM(cfg).to(dtype)
    with torch.no_grad():
        for p, t in zip(m.parameters(), tensors):
            p.copy_(t)
    return m


def _write_outer_optim(path, bufs, lr=0.7, momentum=0.9, nesterov=True):
    ps = [torch.nn.Parameter(b.clone()) for b in bufs]
    opt = torch.optim.SGD(ps, lr=lr, momentum=momentum, nesterov=nesterov)
    for p, b in zip(ps, bufs):
        opt.state[p]["momentum_buffer"] = b.clone()
    torch.save(opt.state_dict(), path)


def gen_pair_merge(manifest, tensors):
    lm = _load_module("ref_lm_crossover", "EDT_LM/train/crossover.py")
    cases = []
    # (name, generation tag, optim files present (p1, p2), run_sgd hyperparams, base regime)
    variants = [
        ("gen0_fresh", "Gen0000", (False, False), (0.7, 0.9, True), "bf16"),
        ("p1_only", "Gen0003", (True, False), (0.7, 0.9, True), "bf16"),
        ("p2_only", "Gen0003", (False, True), (0.7, 0.9, True), "bf16"),
        ("both_parent1_rule", "Gen0003", (True, True), (0.7, 0.9, True), "bf16"),
        ("both_sig_defaults", "Gen0003", (True, True), (0.7, 0.0, False), "bf16"),
        ("gen0_sig_defaults", "Gen0000", (False, False), (0.7, 0.0, False), "bf16"),
        ("gen0_fresh_f32base", "Gen0000", (False, False), (0.7, 0.9, True), "f32"),
        ("p1_only_f32base", "Gen0003", (True, False), (0.7, 0.9, True), "f32"),
    ]
    seed = 5000
    for name, gtag, (has1, has2), (lr, mu, nest), base_regime in variants:
        seed += 1
        gen = torch.Generator().manual_seed(seed)
        cfg = _tiny_llama_config("bfloat16")
        shapes = [p.shape for p in _llama_with(cfg, [], torch.bfloat16).parameters()]
        b1 = [(torch.randn(s, generator=gen) * 0.02).bfloat16() for s in shapes]
        b2 = [(torch.randn(s, generator=gen) * 0.02).bfloat16() for s in shapes]
        m1 = [(b.float() + torch.randn(b.shape, generator=gen) * 1e-3).bfloat16() for b in b1]
        m2 = [(b.float() + torch.randn(b.shape, generator=gen) * 1e-3).bfloat16() for b in b2]
        bdt = torch.float32 if base_regime == "f32" else torch.bfloat16
        buf1 = [(torch.randn(s, generator=gen) * 1e-3).to(bdt) for s in shapes]
        buf2 = [(torch.randn(s, generator=gen) * 1e-3).to(bdt) for s in shapes]
        with tempfile.TemporaryDirectory() as tmp:
            p1 = os.path.join(tmp, "m1", gtag)
            p2 = os.path.join(tmp, "m2", gtag)
            out = os.path.join(tmp, "child", "Gen0004")
            for d in (p1, p2, out):
                os.makedirs(d)
            if has1:
                _write_outer_optim(os.path.join(p1, "outer_optim.pt"), buf1)
            if has2:
                _write_outer_optim(os.path.join(p2, "outer_optim.pt"), buf2)
            mb1 = _llama_with(cfg, b1, torch.bfloat16)
            mb2 = _llama_with(cfg, b2, torch.bfloat16)
            mm1 = _llama_with(cfg, m1, torch.bfloat16)
            mm2 = _llama_with(cfg, m2, torch.bfloat16)
            if base_regime == "f32":
                # transformers 4.x: from_config(model_1.config) builds an fp32 model
                mb1.config = copy.deepcopy(mb1.config)
                mb1.config.dtype = torch.float32
            base = lm.run_linear_merge_5050(mb1, mb2, None, None, out)
            merged_base = [p.detach().clone() for p in base.parameters()]
            lm.run_sgd(mm1, mm2, base, out, p1, p2, lr=lr, momentum=mu, nesterov=nest)
            theta = [p.detach().clone() for p in base.parameters()]
            sd = torch.load(os.path.join(out, "outer_optim.pt"), map_location="cpu", weights_only=True)
            out_bufs = [sd["state"][i].get("momentum_buffer") if i in sd["state"] else None
                        for i in range(len(theta))]
            group = {k: v for k, v in sd["param_groups"][0].items() if k != "params"}
        pre = f"pair_merge/{name}"
        for tag, lst in (("b1", b1), ("b2", b2), ("m1", m1), ("m2", m2), ("buf1", buf1),
                         ("buf2", buf2), ("merged_base", merged_base), ("out_theta", theta)):
            for i, t in enumerate(lst):
                tensors[f"{pre}/{tag}/{i}"] = t
        has_out_buf = out_bufs[0] is not None
        if has_out_buf:
            for i, t in enumerate(out_bufs):
                tensors[f"{pre}/out_buf/{i}"] = t
        cases.append({
            "name": pre, "source": "EDT_LM/train/crossover.py:150-237", "generation": gtag,
            "parent1_optim": has1, "parent2_optim": has2, "call_lr": lr, "call_momentum": mu,
            "call_nesterov": nest, "base_dtype": base_regime, "model_dtype": "bf16",
            "n_tensors": len(shapes), "shapes": [list(s) for s in shapes],
            "has_out_buf": has_out_buf, "saved_param_group": {k: v for k, v in group.items()},
        })
    # uniform_dna_crossover with the global numpy RNG (EDT_LM/train/crossover.py:318-321)
    dna = []
    for seed in (0, 1, 7, 123):
        np.random.seed(seed)
        d1, d2 = [0, 1, 2], [3, 2, 1]
        res = [lm.uniform_dna_crossover(d1, d2) for _ in range(4)]
        dna.append({"seed": seed, "dna1": d1, "dna2": d2, "draws": res})
    manifest["pair_merge"] = cases
    manifest["dna_crossover"] = dna
    # the "no parent optimiser and not generation 0" error (EDT_LM/train/crossover.py:226-227)
    manifest["pair_merge_errors"] = [{"generation": "Gen0003", "parent1_optim": False,
                                      "parent2_optim": False, "raises": "NotImplementedError"}]


# ----------------------------------------------------------------------------------------
# SLERP (EDT_RL/crossover.py:11-81, EDT_EVOMERGE/train/crossover.py:14-83)

def _slerp_inputs(gen):
    cases = []
    shape = (23, 19)
    v0 = torch.randn(shape, generator=gen) * 0.02
    cases.append(("generic", v0, v0 + torch.randn(shape, generator=gen) * 0.02 * 0.05))
    cases.append(("far", v0, torch.randn(shape, generator=gen) * 0.02))
    cases.append(("parallel", v0, 2.0 * v0))
    cases.append(("antiparallel", v0, -v0))
    cases.append(("zero_v0", torch.zeros(shape), v0))
    cases.append(("both_zero", torch.zeros(shape), torch.zeros(shape)))
    cases.append(("single", torch.tensor([0.37]), torch.tensor([-0.11])))
    big = torch.randn(2053, generator=gen) * 0.02
    cases.append(("long", big, big + torch.randn(2053, generator=gen) * 0.01))
    # near the 0.9995 DOT_THRESHOLD on both sides: tune the noise scale for cos ~ 0.9994 / 0.9996
    noise = torch.randn(shape, generator=gen)
    noise = noise - (noise * v0).sum() / (v0 * v0).sum() * v0        # orthogonal to v0
    for tag, target in (("near_below", 0.9994), ("near_above", 0.9996)):
        tan = float(np.sqrt(1.0 / target ** 2 - 1.0))
        cases.append((tag, v0, v0 + noise * (tan * v0.norm() / noise.norm())))
    return cases


def gen_slerp(manifest, tensors):
    rl = _load_module("ref_rl_crossover", "EDT_RL/crossover.py")
    ev = _load_module("ref_ev_crossover", "EDT_EVOMERGE/train/crossover.py")
    gen = torch.Generator().manual_seed(777)
    cases = []
    ts = [0.0, 0.43333333333333335, 0.5, 0.5666666666666667, 1.0]
    for tag, v0, v1 in _slerp_inputs(gen):
        for in_dt in ("f32", "bf16"):
            a = v0.to(DTYPES[in_dt])
            b = v1.to(DTYPES[in_dt])
            n0 = np.linalg.norm(a.float().numpy())
            n1 = np.linalg.norm(b.float().numpy())
            dot = float(np.sum(rl.normalize(a.float().numpy(), 1e-8) * rl.normalize(b.float().numpy(), 1e-8)))
            inp = f"slerp_in/{tag}_{in_dt}"
            tensors[f"{inp}/v0"] = a.contiguous()
            tensors[f"{inp}/v1"] = b.contiguous()
            for j, t in enumerate(ts):
                res = rl.slerp(t, a, b)
                res_ev = ev.slerp(t, a, b)
                assert torch.equal(res, res_ev), "EDT_RL and EDT_EVOMERGE slerp disagree"
                name = f"slerp/{tag}_{in_dt}_t{j}"
                tensors[f"{name}/out"] = res.contiguous()
                cases.append({"name": name, "inputs": inp, "t": t, "in_dtype": in_dt, "ref_dot": dot,
                              "ref_norm0": float(n0), "ref_norm1": float(n1),
                              "lerp_branch": bool(abs(dot) > 0.9995),
                              "source": "EDT_RL/crossover.py:11-43"})
    manifest["slerp"] = cases
    curves = {"self_attn": [0, 0.5, 0.3, 0.7, 1], "mlp": [1, 0.5, 0.7, 0.3, 0]}
    tables = []
    for L in (1, 2, 4, 5, 28):
        for cname, curve in curves.items():
            vals = [rl.interpolate_t(i, L, curve) for i in range(-1, L + 1)]
            vals_ev = [ev.interpolate_t(i, L, curve) for i in range(-1, L + 1)]
            assert vals == vals_ev
            tables.append({"num_layers": L, "curve": cname, "t_curve": curve,
                           "layer_idx": list(range(-1, L + 1)), "t": vals})
    manifest["interpolate_t"] = tables


def gen_merge_models(manifest, tensors):
    """Whole-model SLERP merges: the RL `crossover(g1, g2, out)` over Policy+Value folders and the
    EVOMERGE `run_slerp_merge_from_config` over bf16 Qwen2 bodies."""
    from transformers import LlamaForCausalLM, Qwen2Config, Qwen2ForCausalLM
    rl = _load_module("ref_rl_crossover", "EDT_RL/crossover.py")
    ev = _load_module("ref_ev_crossover", "EDT_EVOMERGE/train/crossover.py")
    out_cases = []
    gen = torch.Generator().manual_seed(4242)

    def rand_llama(noise_from=None):
        cfg = _tiny_llama_config("float32")
        m = LlamaForCausalLM(cfg)
        with torch.no_grad():
            for i, p in enumerate(m.parameters()):
                base = torch.randn(p.shape, generator=gen) * 0.02
                if noise_from is not None:
                    src = list(noise_from.parameters())[i].detach()
                    base = src + torch.randn(p.shape, generator=gen) * 0.02 * 0.05
                p.copy_(base)
        return m

    with tempfile.TemporaryDirectory() as tmp:
        g = {}
        pol1 = rand_llama()
        pol2 = rand_llama(noise_from=pol1)     # related parents -> slerp branch
        val1 = rand_llama()
        val2 = rand_llama()                    # unrelated parents
        for tag, pol, val in (("g1", pol1, val1), ("g2", pol2, val2)):
            root = os.path.join(tmp, tag)
            pol.save_pretrained(os.path.join(root, "Policy"))
            val.save_pretrained(os.path.join(root, "Value"))
            g[tag] = {"model_path": root, "env": {"env_name": "wb", "reward_dna": [1, 2, 3, 4, 5, 6],
                                                  "agents": []}}
        g["g2"]["env"]["reward_dna"] = [6, 5, 4, 3, 2, 1]
        np.random.seed(31)
        out_root = os.path.join(tmp, "child")
        genome = rl.crossover(g["g1"], g["g2"], out_root)
        rec = {"name": "rl_crossover", "source": "EDT_RL/crossover.py:84-201", "np_seed": 31,
               "reward_dna": genome["env"]["reward_dna"], "parts": {}}
        for part in ("Policy", "Value"):
            sd1 = load_file(os.path.join(tmp, "g1", part, "model.safetensors"))
            sd2 = load_file(os.path.join(tmp, "g2", part, "model.safetensors"))
            sdo = load_file(os.path.join(out_root, part, "model.safetensors"))
            keys = sorted(sdo.keys())
            for k in keys:   # parents were saved as *ForCausalLM: body keys carry "model."
                tensors[f"merge_models/rl/{part}/p1/{k}"] = sd1["model." + k]
                tensors[f"merge_models/rl/{part}/p2/{k}"] = sd2["model." + k]
                tensors[f"merge_models/rl/{part}/out/{k}"] = sdo[k]
            rec["parts"][part] = {"keys": keys, "num_hidden_layers": 4,
                                  "p1_keys": sorted(sd1.keys())}
        out_cases.append(rec)

        # EVOMERGE: bf16 Qwen2 bodies, result written into model_1 (bf16)
        qcfg = Qwen2Config(vocab_size=24, hidden_size=8, intermediate_size=16, num_hidden_layers=5,
                           num_attention_heads=2, num_key_value_heads=1, tie_word_embeddings=False)
        q1 = Qwen2ForCausalLM(qcfg)
        q2 = Qwen2ForCausalLM(qcfg)
        with torch.no_grad():
            for p1_, p2_ in zip(q1.parameters(), q2.parameters()):
                a = torch.randn(p1_.shape, generator=gen) * 0.02
                p1_.copy_(a)
                p2_.copy_(a + torch.randn(p1_.shape, generator=gen) * 0.02 * 0.05)
        q1 = q1.to(torch.bfloat16)
        q2 = q2.to(torch.bfloat16)
        p1_sd = {k: v.clone() for k, v in q1.model.state_dict().items()}
        p2_sd = {k: v.clone() for k, v in q2.model.state_dict().items()}
        lm_head = q1.lm_head.weight.detach().clone()
        merge_cfg = {"slices": [{"sources": [{"model": "a", "layer_range": [0, 5]},
                                             {"model": "b", "layer_range": [0, 5]}]}],
                     "merge_method": "slerp", "base_model": "a",
                     "parameters": {"t": [{"filter": "self_attn", "value": [0, 0.5, 0.3, 0.7, 1]},
                                          {"filter": "mlp", "value": [1, 0.5, 0.7, 0.3, 0]},
                                          {"value": 0.5}]},
                     "dtype": "float32", "tokenizer_source": None}
        ev.run_slerp_merge_from_config(merge_cfg, q1.model, q2.model, qcfg, qcfg,
                                       os.path.join(tmp, "evo_out"), base_model=q1, device="cpu")
        keys = sorted(p1_sd.keys())
        for k in keys:
            tensors[f"merge_models/evomerge/p1/{k}"] = p1_sd[k]
            tensors[f"merge_models/evomerge/p2/{k}"] = p2_sd[k]
            tensors[f"merge_models/evomerge/out/{k}"] = q1.model.state_dict()[k].clone()
        tensors["merge_models/evomerge/out_lm_head"] = q1.lm_head.weight.detach().clone()
        assert torch.equal(lm_head, tensors["merge_models/evomerge/out_lm_head"])
        out_cases.append({"name": "evomerge", "source": "EDT_EVOMERGE/train/crossover.py:104-146",
                          "keys": keys, "num_hidden_layers": 5, "model_dtype": "bf16"})
    manifest["merge_models"] = out_cases


# ----------------------------------------------------------------------------------------
# selection (module-level nested defs in the masters: compiled from the source text)

SELECTION_DEFS = {
    "rank_based_lm_sim": ("EDT_LM/edt_sim.py", 177, 214, "rank_based_selection"),
    "rank_based_lm": ("EDT_LM/edt.py", 185, 211, "rank_based_selection"),
    "tournament_lm": ("EDT_LM/edt.py", 213, 224, "tournament_selection"),
    "rank_based_evomerge": ("EDT_EVOMERGE/edt.py", 193, 230, "rank_based_selection"),
    "roulette_rl": ("EDT_RL/edt.py", 221, 240, "roulette_wheel_selection"),
    "rank_based_rl": ("EDT_RL/edt.py", 243, 261, "rank_based_selection"),
}


def gen_selection(manifest, tensors):
    import random
    recs = []
    genomes = [{"model_path": f"m{i}/Gen0003", "fitness": f, "dna": [i % 4, 1, 2]}
               for i, f in enumerate([0.31, 0.52, 0.18, 0.52, 0.77, 0.05, 0.44, 0.29])]
    for name, (rel, first, last, fn) in SELECTION_DEFS.items():
        ns = {"random": random, "YELLOW": "", "RESET": "", "print": lambda *a, **k: None}
        exec(_block(rel, first, last), ns)
        f = ns[fn]
        for seed in (0, 3, 11):
            for num_pairs in (1, 4, 7):
                args = (genomes, num_pairs)
                extra = []
                if name == "roulette_rl":
                    for scale in (0.1, 1.3, 2.5):
                        random.seed(seed)
                        pairs = f(genomes, num_pairs, scale)
                        recs.append({"fn": name, "source": f"{rel}:{first}-{last}", "seed": seed,
                                     "num_pairs": num_pairs, "scale": scale,
                                     "pairs": [[genomes.index(a), genomes.index(b)] for a, b in pairs]})
                    continue
                random.seed(seed)
                pairs = f(*args, *extra)
                recs.append({"fn": name, "source": f"{rel}:{first}-{last}", "seed": seed, "num_pairs": num_pairs,
                             "pairs": [[genomes.index(a), genomes.index(b)] for a, b in pairs]})
    manifest["selection"] = {"genomes": genomes, "cases": recs}


def main():
    torch.manual_seed(0)
    manifest = {"generated_with": {"torch": torch.__version__, "numpy": np.__version__}}
    import transformers
    manifest["generated_with"]["transformers"] = transformers.__version__
    for fn, fname in ((gen_diloco, "diloco"), (gen_pair_merge, "pair_merge"),
                      (gen_slerp, "slerp"), (gen_merge_models, "merge_models"), (gen_selection, None)):
        tensors = {}
        fn(manifest, tensors)
        if fname is None:
            continue
        tensors = {k: v.detach().contiguous().clone() for k, v in tensors.items()}
        save_file(tensors, os.path.join(HERE, f"{fname}.safetensors"))
        print(f"{fname}: {len(tensors)} tensors")
    with open(os.path.join(HERE, "manifest.json"), "w") as f:
        json.dump(manifest, f, indent=1)


if __name__ == "__main__":
    main()
