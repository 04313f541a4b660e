"""Drop-in for EDT_RL/crossover.py: SLERP crossover of Policy/Value models, run in-process by the
RL master (EDT_RL/edt.py:6 imports `crossover`, :290 calls it once per selected pair).

Same functions, arguments, return values and files as the reference; the per-key numpy loop is
replaced by one multi-tensor SLERP on the GPU (merge.slerp_state_dicts).
"""
from __future__ import annotations

import os

from .merge import (interpolate_t, lerp, maybe_torch, merge_plan, normalize, slerp,  # noqa: F401
                    slerp_state_dicts, uniform_dna_crossover)

__all__ = ["slerp", "lerp", "interpolate_t", "load_model_from_folder", "run_slerp_merge_from_config",
           "run_slerp_merge", "uniform_crossover", "crossover", "SELF_ATTN_T_CURVE", "MLP_T_CURVE", "maybe_torch", "normalize"]

# hard-coded layer curves of run_slerp_merge (EDT_RL/crossover.py:146-147)
SELF_ATTN_T_CURVE = [0, 0.5, 0.3, 0.7, 1]
MLP_T_CURVE = [1, 0.5, 0.7, 0.3, 0]


def load_model_from_folder(folder_path: str):
    """AutoModel.from_pretrained(trust_remote_code=True), placed on the GPU (EDT_RL/crossover.py:63-67)."""
    import torch
    from transformers import AutoConfig, AutoModel
    config = AutoConfig.from_pretrained(folder_path, trust_remote_code=True)
    model = AutoModel.from_pretrained(folder_path, config=config, trust_remote_code=True)
    return model.to(torch.device("cuda", torch.cuda.current_device()))


def run_slerp_merge_from_config(merge_config_dict: dict, merge_output_path: str) -> str:
    """SLERP two model folders named by a MergeKit-style config (EDT_RL/crossover.py:84-135)."""
    from transformers import AutoConfig, AutoModel
    sources = merge_config_dict["slices"][0]["sources"]
    path_1, path_2 = sources[0]["model"], sources[1]["model"]
    model_1 = load_model_from_folder(path_1)
    model_2 = load_model_from_folder(path_2)
    config_1 = AutoConfig.from_pretrained(path_1, trust_remote_code=True)
    config_2 = AutoConfig.from_pretrained(path_2, trust_remote_code=True)
    num_layers = min(config_1.num_hidden_layers, config_2.num_hidden_layers)
    merged_model = AutoModel.from_config(model_1.config, trust_remote_code=True)
    sd1, sd2 = model_1.state_dict(), model_2.state_dict()
    plan = merge_plan(list(sd1.keys()), num_layers, merge_config_dict)
    merged = slerp_state_dicts(sd1, sd2, plan)
    merged_model.load_state_dict(merged)
    merged_model.save_pretrained(merge_output_path)
    print("SLERP merging complete! Model saved at:", merge_output_path)
    return merge_output_path


def run_slerp_merge(p1_folder: str, p2_folder: str, output_path: str) -> None:
    """SLERP with the RL layer curves (EDT_RL/crossover.py:138-164)."""
    import json
    with open(os.path.join(p1_folder, "config.json")) as f:
        l1 = json.load(f)["num_hidden_layers"]
    with open(os.path.join(p2_folder, "config.json")) as f:
        l2 = json.load(f)["num_hidden_layers"]
    num_layers = min(l1, l2)
    cfg = {
        "slices": [{"sources": [{"model": p1_folder, "layer_range": [0, num_layers]},
                                {"model": p2_folder, "layer_range": [0, num_layers]}]}],
        "merge_method": "slerp", "base_model": p1_folder,
        "parameters": {"t": [{"filter": "self_attn", "value": SELF_ATTN_T_CURVE},
                             {"filter": "mlp", "value": MLP_T_CURVE}, {"value": 0.5}]},
        "dtype": "float32", "tokenizer_source": None,
    }
    run_slerp_merge_from_config(cfg, output_path)
    print("Done!")


def uniform_crossover(dna1, dna2):
    """Reward-DNA uniform crossover (EDT_RL/crossover.py:167-170)."""
    return uniform_dna_crossover(dna1, dna2)


def crossover(g1: dict, g2: dict, output_path: str) -> dict:
    """Child genome of two RL genomes: SLERP of Policy and Value, uniform reward-DNA crossover
    (EDT_RL/crossover.py:173-201). The caller fills `agents` and writes genome.json."""
    run_slerp_merge(os.path.join(g1["model_path"], "Policy"), os.path.join(g2["model_path"], "Policy"),
                    os.path.join(output_path, "Policy"))
    run_slerp_merge(os.path.join(g1["model_path"], "Value"), os.path.join(g2["model_path"], "Value"),
                    os.path.join(output_path, "Value"))
    reward_dna = uniform_crossover(g1["env"]["reward_dna"], g2["env"]["reward_dna"])
    return {
        "model_path": output_path,
        "env": {"env_name": g1["env"]["env_name"], "reward_dna": reward_dna, "agents": []},
        "p1": g1,
        "p2": g2,
    }
