"""A single-process DiLoCo simulation on one MI355X with this package's outer step — the shape of
the reference's EDT_LM/diloco_sim.py (K simulated workers, each training a copy of the global
model for an inner phase, then the master's outer step, EDT_LM/diloco.py:238-289), with the
inner training done in-process on synthetic tokens instead of TRL SFT over a shared disk.

The outer step is `diloco.outer_step(base_params, worker_params, state, lr, momentum, nesterov)`:
one fused HIP launch over the tensor lists (no packing), the outer momentum carried in `state`
exactly as the reference's `outer_optimizer.load_state_dict` carry.

    python examples/diloco_sim.py [--generations 5 --workers 4 --inner-steps 20]
"""
from __future__ import annotations

import argparse
import copy
import os
import sys

import torch
import torch.nn as nn

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

VOCAB, CTX = 256, 64


class TinyLM(nn.Module):
    """A small causal transformer LM (the reference's sims use a tiny GPT-2 / Llama)."""

    def __init__(self, d: int = 64, layers: int = 2, heads: int = 4):
        super().__init__()
        self.tok = nn.Embedding(VOCAB, d)
        self.pos = nn.Embedding(CTX, d)
        layer = nn.TransformerEncoderLayer(d, heads, 4 * d, dropout=0.0, batch_first=True, norm_first=True)
        self.blocks = nn.TransformerEncoder(layer, layers, enable_nested_tensor=False)
        self.head = nn.Linear(d, VOCAB)

    def forward(self, x):
        n = x.shape[1]
        h = self.tok(x) + self.pos(torch.arange(n, device=x.device))
        mask = nn.Transformer.generate_square_subsequent_mask(n, device=x.device)
        return self.head(self.blocks(h, mask=mask, is_causal=True))


def batch(seed: int, device, size: int = 16) -> torch.Tensor:
    """Synthetic sequences with a learnable rule: x[i+1] = (3 x[i] + 1) mod VOCAB."""
    g = torch.Generator(device="cpu").manual_seed(seed)
    x0 = torch.randint(0, VOCAB, (size, 1), generator=g)
    seq = [x0]
    for _ in range(CTX - 1):
        seq.append((3 * seq[-1] + 1) % VOCAB)
    return torch.cat(seq, 1).to(device)


def loss_of(model, x):
    logits = model(x[:, :-1])
    return nn.functional.cross_entropy(logits.reshape(-1, VOCAB), x[:, 1:].reshape(-1))


def inner_train(model, worker: int, gen: int, steps: int, device, lr: float = 3e-3) -> float:
    """The worker's inner phase (the reference runs TRL SFT here): AdamW on its own data."""
    opt = torch.optim.AdamW(model.parameters(), lr=lr)
    last = 0.0
    for s in range(steps):
        x = batch(10_000 * gen + 100 * worker + s, device)
        loss = loss_of(model, x)
        opt.zero_grad(set_to_none=True)
        loss.backward()
        opt.step()
        last = float(loss.detach())
    return last


def run(generations: int = 5, workers: int = 4, inner_steps: int = 20, device="cuda", seed: int = 0,
        before_outer=None, after_outer=None, log=print):
    """The simulation loop. before_outer(gen, base, replicas) / after_outer(gen, base, state) are
    hooks (the tests snapshot and check the outer step there). Returns the eval losses."""
    from evolutionarydistributedtraining_amd import diloco
    torch.manual_seed(seed)
    device = torch.device(device)
    base = TinyLM().to(device)
    state = None
    evals = []
    for gen in range(generations):
        replicas = []
        for k in range(workers):                     # every worker starts from the global model
            m = copy.deepcopy(base)
            inner_train(m, k, gen, inner_steps, device)
            replicas.append(m)
        if before_outer:
            before_outer(gen, base, replicas)
        with torch.no_grad():
            state = diloco.outer_step(list(base.parameters()), [list(m.parameters()) for m in replicas], state,
                                      lr=0.7, momentum=0.9, nesterov=True)
        if after_outer:
            after_outer(gen, base, state)
        with torch.no_grad():
            ev = float(loss_of(base, batch(999_999, device, 64)))
        evals.append(ev)
        log(f"generation {gen}: eval loss {ev:.4f}")
    return evals


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--generations", type=int, default=5)
    ap.add_argument("--workers", type=int, default=4)
    ap.add_argument("--inner-steps", type=int, default=20)
    a = ap.parse_args()
    run(a.generations, a.workers, a.inner_steps)


if __name__ == "__main__":
    main()
