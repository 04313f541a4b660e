"""Loader for the committed golden vectors (tests/golden/*.safetensors + manifest.json).

The vectors were produced by the reference's own code by tests/golden/gen_golden.py; this module
only reads them (safetensors: no code execution) and never touches /root/reference.
"""
from __future__ import annotations

import json
import os

import torch
from safetensors.torch import load_file

GOLDEN_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


class Golden:
    def __init__(self, root: str = GOLDEN_DIR):
        with open(os.path.join(root, "manifest.json")) as f:
            self.manifest = json.load(f)
        self._files = {}
        self.root = root

    def tensors(self, section: str) -> dict[str, torch.Tensor]:
        if section not in self._files:
            self._files[section] = load_file(os.path.join(self.root, f"{section}.safetensors"))
        return self._files[section]

    def tlist(self, section: str, prefix: str, count: int) -> list[torch.Tensor]:
        t = self.tensors(section)
        return [t[f"{prefix}/{i}"] for i in range(count)]

    def diloco_cases(self):
        return self.manifest["diloco"]

    def pair_cases(self):
        return self.manifest["pair_merge"]

    def slerp_cases(self):
        return self.manifest["slerp"]


def flat(tensors: list[torch.Tensor]) -> torch.Tensor:
    return torch.cat([t.reshape(-1) for t in tensors]) if tensors else torch.empty(0)


def bits(t: torch.Tensor) -> torch.Tensor:
    """Integer view for bit-exact comparison (NaN-safe, sign-of-zero-safe)."""
    return t.contiguous().view(torch.int16 if t.dtype == torch.bfloat16 else torch.int32)
