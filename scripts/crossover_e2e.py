"""End-to-end EDT-LM crossover (the worker CLI, EDT_LM/train/crossover.py:240-315) on a
125M-class Llama: four parent checkpoints on local disk -> child checkpoint, timed with the
parents read straight into HBM arenas (crossover_main(direct=True)) and through four
`from_pretrained` loads (direct=False). Page cache warm (the parents were just written).

    python scripts/crossover_e2e.py [--dir /tmp/xo] [--reps 2]
"""
from __future__ import annotations

import argparse
import json
import os
import shutil
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def _save_tokenizer(path):
    from tokenizers import Tokenizer, models, pre_tokenizers
    from transformers import PreTrainedTokenizerFast
    vocab = {"[UNK]": 0, **{f"w{i}": i + 1 for i in range(23)}}
    tok = Tokenizer(models.WordLevel(vocab, unk_token="[UNK]"))
    tok.pre_tokenizer = pre_tokenizers.Whitespace()
    PreTrainedTokenizerFast(tokenizer_object=tok, unk_token="[UNK]").save_pretrained(path)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--dir", default="/tmp/edt_xo")
    ap.add_argument("--reps", type=int, default=2)
    a = ap.parse_args()
    from transformers import LlamaConfig, LlamaForCausalLM
    from evolutionarydistributedtraining_amd import lm_crossover
    dev = torch.device("cuda:0")
    cfg = LlamaConfig(vocab_size=32000, hidden_size=768, intermediate_size=3072, num_hidden_layers=12,
                      num_attention_heads=12, num_key_value_heads=12, tie_word_embeddings=False)
    shutil.rmtree(a.dir, ignore_errors=True)
    dirs = {}
    for tag in ("1", "2"):
        for kind in ("base", "mut"):
            with torch.device(dev):
                m = LlamaForCausalLM(cfg).to(torch.bfloat16)
            d = os.path.join(a.dir, f"m{tag}", "Gen0000" if kind == "base" else "Gen0000_mutation")
            m.save_pretrained(d)
            dirs[(tag, kind)] = d
            del m
            if kind == "mut":
                _save_tokenizer(d)
        with open(os.path.join(dirs[(tag, "base")], "genome.json"), "w") as f:
            json.dump({"fitness": 1.0, "model_path": dirs[(tag, "base")], "dna": [0, 1, 2],
                       "mutation_path": dirs[(tag, "mut")]}, f)
    n_params = sum(p.numel() for p in LlamaForCausalLM(cfg).parameters())
    res = {"params": n_params, "dtype": "bf16"}
    for direct in (True, False):
        ts = []
        for r in range(a.reps):
            out = os.path.join(a.dir, f"child_{int(direct)}_{r}")
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            lm_crossover.crossover_main(dirs[("1", "base")], dirs[("2", "base")], out, direct=direct)
            torch.cuda.synchronize()
            ts.append(time.perf_counter() - t0)
        res["direct" if direct else "from_pretrained"] = {"s": [round(t, 3) for t in ts]}
    print(json.dumps(res))


if __name__ == "__main__":
    main()
