"""Deterministic inputs of the SLERP branch-threshold fixtures (tests/golden/slerp_threshold.*).

Shared by the generator (gen_slerp_threshold.py, run once in the build container against the
reference) and the tests, which rebuild the large inputs from their seed and noise scale instead of
storing megabytes: torch's CPU generator, fp64 element-wise ops and an RNE cast are deterministic,
and the tests check a SHA-256 of the rebuilt bytes against the one recorded at generation time.
No reference code here."""
from __future__ import annotations

import hashlib

import torch

DTYPES = {"f32": torch.float32, "bf16": torch.bfloat16}


def make_pair(seed: int, n: int, dtype: str, s: float):
    """v0 ~ N(0, .02^2); v1 = v0 + s * .02 * noise, both computed in fp64 and rounded to dtype."""
    g = torch.Generator().manual_seed(seed)
    v0 = torch.randn(n, generator=g, dtype=torch.float64) * 0.02
    noise = torch.randn(n, generator=g, dtype=torch.float64)
    v1 = v0 + (s * 0.02) * noise
    return v0.to(DTYPES[dtype]), v1.to(DTYPES[dtype])


def digest(a: torch.Tensor, b: torch.Tensor) -> str:
    h = hashlib.sha256()
    for t in (a, b):
        h.update(t.contiguous().view(torch.uint8).numpy().tobytes())
    return h.hexdigest()


def exact_cos(a: torch.Tensor, b: torch.Tensor) -> float:
    """cos(a, b) of the rounded vectors in fp64 (fsum-accurate enough for 1e-9 targeting)."""
    x, y = a.double(), b.double()
    return float((x * y).sum() / (x.norm() * y.norm()))


def sample_index(n: int, k: int = 4096) -> torch.Tensor:
    """The output elements a large case records (every element for small ones)."""
    if n <= k:
        return torch.arange(n)
    g = torch.Generator().manual_seed(n)
    return torch.sort(torch.randperm(n, generator=g)[:k]).values
