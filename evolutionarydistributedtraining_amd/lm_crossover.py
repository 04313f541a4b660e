"""Drop-in for EDT_LM/train/crossover.py: the EDT pairwise SGD-merge, run on a worker by
EDT_LM/edt.py:264-280 / edt_sim.py:246-256 through the CLI

    python -m evolutionarydistributedtraining_amd.lm_crossover --model1_path A --model2_path B --output_path O

Child of parents A, B (their pre-training dirs; `genome.json` names the trained `mutation_path`):
    B0 = lerp(0.5, base_A, base_B)                             run_linear_merge_5050 (:150-163)
    d  = ((trained_A - B0) + (trained_B - B0)) / 2; grad = -d   run_sgd (:166-181)
    SGD(lr .7, momentum .9, nesterov).step() with parent A's outer momentum (:183-230)
crossover_main fuses the two into ONE HIP launch over flat parameter arenas (edt_pair_merge):
every parent tensor is read once, the child and its momentum written once.
"""
from __future__ import annotations

import json
import os
import shutil

import torch

from . import ops
from ._lib import EdtError
from .diloco import OuterState, check_sgd_hparams
from .evomerge_crossover import run_slerp_merge_from_config  # noqa: F401  (same surface as :105-147)
from .merge import LazyTensorLoader, interpolate_t, lerp, maybe_torch, normalize, slerp, uniform_dna_crossover  # noqa: F401
from .params import ParamLayout, flat_view, pack, unpack_

__all__ = ["lerp", "slerp", "interpolate_t", "load_model_from_path", "run_slerp_merge_from_config",
           "run_linear_merge_5050", "run_sgd", "crossover_main", "uniform_dna_crossover",
           "load_parent_outer_state", "LazyTensorLoader", "maybe_torch", "normalize"]

# hyper-parameter tables of the DNA (EDT_LM/train/crossover.py:286-294). The reference picks
# entries 0 / 1 / -1 regardless of the DNA: lr 0.7, momentum 0.9, nesterov True.
LR_SETTINGS = [0.7, 0.8, 0.9, 1.0]
MOMENTUM_SETTINGS = [0.7, 0.9, 0.99, 2.00]
NESTEROV_SETTINGS = [False, False, True, True]


def _device():
    return torch.device("cuda", torch.cuda.current_device())


def load_model_from_path(folder_path: str):
    """bf16 AutoModelForCausalLM on the GPU (EDT_LM/train/crossover.py:67-70)."""
    from transformers import AutoConfig, AutoModelForCausalLM
    config = AutoConfig.from_pretrained(folder_path, trust_remote_code=True, cache_dir="cache")
    model = AutoModelForCausalLM.from_pretrained(folder_path, config=config, torch_dtype=torch.bfloat16,
                                                 trust_remote_code=True, cache_dir="cache")
    return model.to(_device())


def run_linear_merge_5050(model_1, model_2, config_1, config_2, merge_output_path):
    """New model from model_1's config holding lerp(0.5) of both state dicts (not saved),
    EDT_LM/train/crossover.py:150-163. The lerp is one launch over the packed state dicts."""
    from transformers import AutoModelForCausalLM
    merged_model = AutoModelForCausalLM.from_config(model_1.config)
    sd1, sd2 = model_1.state_dict(), model_2.state_dict()
    keys = list(sd1.keys())
    dev = next(model_1.parameters()).device
    if dev.type != "cuda":
        dev = _device()
    a = pack([sd1[k] for k in keys], device=dev)
    b = pack([sd2[k] for k in keys], dtype=a.dtype, device=dev)
    out = ops.lerp(0.5, a, b)
    layout = ParamLayout.of([sd1[k] for k in keys])
    merged_model.load_state_dict(dict(zip(keys, layout.views(out))))
    return merged_model.to(dev)


def load_parent_outer_state(model1_path: str, model2_path: str):
    """The outer-optimizer state a child inherits (EDT_LM/train/crossover.py:183-227):
    both parents' outer_optim.pt -> parent 1's per-parameter state (the reference's "merge"
    falls back to the first parent for the nested per-parameter dicts and the param_groups);
    one -> that one; none -> None, an error unless this is generation 0."""
    p1 = os.path.join(model1_path, "outer_optim.pt")
    p2 = os.path.join(model2_path, "outer_optim.pt")
    if os.path.exists(p1) and os.path.exists(p2):
        print(f"Merging outer optimizers: {p1} and {p2}")
        s1 = torch.load(p1, map_location="cpu", weights_only=True)
        s2 = torch.load(p2, map_location="cpu", weights_only=True)
        merged = {}
        for k in list(s1) + [k for k in s2 if k not in s1]:
            if k in s1 and k in s2 and isinstance(s1[k], dict) and isinstance(s2[k], dict):
                # tensors present in both are averaged; anything else (the per-parameter
                # {"momentum_buffer": ...} dicts of an SGD state) is parent 1's; parent 2 fills gaps
                sub = {}
                for sk, v1 in s1[k].items():
                    v2 = s2[k].get(sk)
                    both = sk in s2[k] and torch.is_tensor(v1) and torch.is_tensor(v2)
                    sub[sk] = (v1 + v2) / 2 if both else v1
                for sk, v2 in s2[k].items():
                    sub.setdefault(sk, v2)
                merged[k] = sub
            elif k in s1 and k in s2 and torch.is_tensor(s1[k]) and torch.is_tensor(s2[k]):
                merged[k] = (s1[k] + s2[k]) / 2
            else:
                merged[k] = s1[k] if k in s1 else s2[k]
        return merged
    if os.path.exists(p1):
        print(f"Loading outer optimizer: {p1}")
        return torch.load(p1, map_location="cpu", weights_only=True)
    if os.path.exists(p2):
        print(f"Loading outer optimizer: {p2}")
        return torch.load(p2, map_location="cpu", weights_only=True)
    if "0000" not in p1:
        raise NotImplementedError(f"What, no {p1} or {p2}?")
    return None


def _child_step(b1, b2, m1, m2, base_params, layout, state_sd, lr, momentum, nesterov, output_path):
    """Shared body of run_sgd / crossover_main: one edt_pair_merge launch, then the outputs."""
    theta = flat_view(base_params)
    copied = theta is None
    if copied:
        theta = pack(base_params, device=m1.device)
    st = OuterState()
    if state_sd is not None:
        st.load_state_dict(state_sd, layout, theta.dtype, theta.device)
        lr, momentum, nesterov = st.hparams["lr"], st.hparams["momentum"], st.hparams["nesterov"]
    check_sgd_hparams(lr, momentum, nesterov)          # optim.SGD(...) at :228-230
    mom = None
    if momentum != 0:
        mom = st.momentum if st.has_momentum else torch.zeros_like(theta)
    out = theta if b1 is None else torch.empty_like(theta)
    src = theta if b1 is None else b1
    ops.pair_merge(src, b2, m1, m2, out, mom, st.has_momentum and momentum != 0, lr, momentum, nesterov)
    if b1 is not None:
        theta.copy_(out)
    if copied:
        unpack_(theta, base_params)
    st.hparams = dict(lr=lr, momentum=momentum, nesterov=nesterov)
    st.momentum, st.has_momentum = (mom, True) if momentum != 0 else (st.momentum, st.has_momentum)
    os.makedirs(output_path, exist_ok=True)
    st.save(os.path.join(output_path, "outer_optim.pt"), layout)


def run_sgd(model_1, model_2, base_model, output_path, model1_path, model2_path, lr=0.7, momentum=0.0,
            nesterov=False):
    """EDT_LM/train/crossover.py:166-237: SGD step of base_model (in place) along the mean of the
    two parents' pseudo-gradients; writes outer_optim.pt and the model to output_path."""
    params1, params2 = list(model_1.parameters()), list(model_2.parameters())
    base_params = list(base_model.parameters())
    if not (len(params1) == len(params2) == len(base_params)):
        raise EdtError("parents and base model have different parameter lists")
    dev = base_params[0].device if base_params[0].is_cuda else _device()
    m1 = flat_view(params1)
    m1 = m1 if m1 is not None and m1.device == dev else pack(params1, device=dev)
    m2 = flat_view(params2)
    m2 = m2 if m2 is not None and m2.device == dev else pack(params2, dtype=m1.dtype, device=dev)
    state_sd = load_parent_outer_state(model1_path, model2_path)
    with torch.no_grad():
        _child_step(None, None, m1, m2, base_params, ParamLayout.of(base_params), state_sd, lr, momentum,
                    nesterov, output_path)
    base_model.save_pretrained(output_path)
    print("SGD merge complete! Model saved at:", output_path)
    return output_path


def _read_parents_direct(paths, dev):
    """The child model (`from_config` of the first trained model's config, bf16, built on the
    GPU) bound to a flat arena, and the four parents' checkpoints read straight into bf16 arenas
    in the child's `parameters()` order (checkpoint.read_into_arena: safetensors -> pinned host
    -> HBM, no model objects). None when a checkpoint lacks one of the child's parameter names
    (the caller then loads the parents with from_pretrained)."""
    from transformers import AutoConfig, AutoModelForCausalLM
    from .checkpoint import checkpoint_files, read_into_arena
    from .params import ParamArena, bind_module_
    config = AutoConfig.from_pretrained(paths[0], trust_remote_code=True, cache_dir="cache")
    config.dtype = torch.bfloat16            # what from_pretrained(torch_dtype=bf16) leaves in model_1.config
    with torch.device(dev):
        child = AutoModelForCausalLM.from_config(config)
    layout = ParamLayout.of_module(child)
    for p in paths:
        try:
            have = checkpoint_files(p)
        except (OSError, ValueError):
            return None
        if any(n not in have for n in layout.names):
            return None
    # the child keeps its own dtype; the parents are always read as bf16, as the reference loads
    # them (from_pretrained(torch_dtype=bf16), :67-70), so lerp(0.5) of the bases rounds to bf16
    # even when from_config builds an fp32 child (the kernel takes bf16 parents + an fp32 child)
    arena = bind_module_(child, ParamArena(layout, next(child.parameters()).dtype, dev), copy=False)
    parents = [read_into_arena(p, layout, torch.empty(layout.total, dtype=torch.bfloat16, device=dev))
               for p in paths]
    return child, arena, parents


def crossover_main(model1_path, model2_path, output_path, direct: bool = True):
    """EDT_LM/train/crossover.py:240-315 with run_linear_merge_5050 + run_sgd fused.

    direct=True reads the four parent checkpoints straight into HBM arenas (SURVEY 8(f)1's I/O
    edge); the results are the same as through from_pretrained (same bf16 conversion)."""
    from transformers import AutoModelForCausalLM, AutoTokenizer
    with open(os.path.join(model1_path, "genome.json")) as f:
        p1_genome = json.load(f)
    with open(os.path.join(model2_path, "genome.json")) as f:
        p2_genome = json.load(f)
    base1_path, base2_path = model1_path, model2_path
    trained1_path, trained2_path = p1_genome.get("mutation_path"), p2_genome.get("mutation_path")

    dev = _device()
    got = _read_parents_direct([trained1_path, trained2_path, base1_path, base2_path], dev) if direct else None
    if got is not None:
        child, _, (m1, m2, b1, b2) = got
    else:
        model_1 = load_model_from_path(trained1_path)
        model_2 = load_model_from_path(trained2_path)
        base_1 = load_model_from_path(base1_path)
        base_2 = load_model_from_path(base2_path)
        child = AutoModelForCausalLM.from_config(model_1.config).to(dev)
        # the state dicts of the bases and parameters() of the trained models share one order
        # for untied HF causal LMs; both sides are packed into flat arenas in parameters() order
        with torch.no_grad():
            b1 = pack(list(base_1.parameters()), device=dev)
            b2 = pack(list(base_2.parameters()), dtype=b1.dtype, device=dev)
            m1 = pack(list(model_1.parameters()), dtype=b1.dtype, device=dev)
            m2 = pack(list(model_2.parameters()), dtype=b1.dtype, device=dev)
        del model_1, model_2, base_1, base_2
    child_params = list(child.parameters())

    tokenizer = AutoTokenizer.from_pretrained(trained1_path, trust_remote_code=True, cache_dir="cache")
    tokenizer.save_pretrained(output_path)
    for fname in ("optimizer.pt", "scheduler.pt"):
        for src in (os.path.join(trained1_path, fname), os.path.join(trained2_path, fname)):
            if os.path.exists(src):
                shutil.copy(src, os.path.join(output_path, fname))
                break

    for g in (p1_genome, p2_genome):
        g.pop("p1", None)
        g.pop("p2", None)
    dna = uniform_dna_crossover(p1_genome["dna"], p2_genome["dna"])
    lr, momentum, nesterov = LR_SETTINGS[0], MOMENTUM_SETTINGS[1], NESTEROV_SETTINGS[-1]
    with open(os.path.join(output_path, "genome.json"), "w") as f:
        json.dump({"fitness": 0.0, "model_path": output_path, "dna": dna, "p1": p1_genome,
                   "p2": p2_genome}, f, indent=4)

    with torch.no_grad():
        state_sd = load_parent_outer_state(base1_path, base2_path)
        _child_step(b1, b2, m1, m2, child_params, ParamLayout.of(child_params), state_sd, lr, momentum,
                    nesterov, output_path)
    child.save_pretrained(output_path)
    print("SGD merge complete! Model saved at:", output_path)
    print("Done!")


def main(argv=None):
    import argparse
    ap = argparse.ArgumentParser(description="SGD merge two Hugging Face models using base models from genome.")
    ap.add_argument("--model1_path", type=str, required=True)
    ap.add_argument("--model2_path", type=str, required=True)
    ap.add_argument("--output_path", type=str, default="crossover_result")
    a = ap.parse_args(argv)
    crossover_main(a.model1_path, a.model2_path, a.output_path)


if __name__ == "__main__":
    main()
