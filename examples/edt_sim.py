"""A single-process EDT-LM simulation on one MI355X with the package's resident population — the
shape of the reference's EDT_LM/edt_sim.py (a population of models; each generation every member
trains, is scored, the master selects parent pairs by rank (edt_sim.py:177-240) and each child is
the pairwise SGD merge of its parents, EDT_LM/train/crossover.py:150-237), with the population kept
in HBM (population.ResidentPopulation) instead of moving through a shared disk, and the inner
training done in-process on the synthetic tokens of examples/diloco_sim.py.

Each member's trained arena is bound to a TinyLM (params.bind_module_): the inner loop's AdamW
updates the arena in place; `pop.step(fitness)` runs selection, the merge kernel for every child
(edt_pair_merge_population: lerp(0.5) of the parents' bases + an SGD step along their mean
pseudo-gradient with the donor's outer momentum) and the swap.

    python examples/edt_sim.py [--generations 4 --population 4 --inner-steps 10 --elitism 1]
"""
from __future__ import annotations

import argparse
import os
import random
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))


def run(generations: int = 4, population: int = 4, inner_steps: int = 10, elitism: int = 1, device="cuda",
        seed: int = 0, before_step=None, after_step=None, log=print):
    """The simulation loop. before_step(gen, pop) / after_step(gen, pop, pairs) are hooks (the
    tests snapshot and check the merge there). Returns the best fitness per generation."""
    from diloco_sim import TinyLM, batch, inner_train, loss_of

    from evolutionarydistributedtraining_amd.params import ParamArena, ParamLayout, bind_module_, pack
    from evolutionarydistributedtraining_amd.population import ResidentPopulation
    random.seed(seed)
    np.random.seed(seed)
    torch.manual_seed(seed)
    device = torch.device(device)
    net = TinyLM().to(device)
    layout = ParamLayout.of_module(net)
    init = pack(net.parameters())                       # Gen0000: every member starts here
    genomes = [{"dna": [random.random() for _ in range(4)]} for _ in range(population)]
    pop = ResidentPopulation(layout, torch.float32, device, genomes, kind="sgd", elitism=elitism)
    for m in range(population):
        pop.base(m).copy_(init)
    best = []
    for gen in range(generations):
        pop.begin_inner()                               # trained = base, then the inner loop
        fitness = []
        for m in range(population):
            bind_module_(net, ParamArena(layout, torch.float32, device, flat=pop.trained(m)), copy=False)
            inner_train(net, m, gen, inner_steps, device)
            with torch.no_grad():
                fitness.append(-float(loss_of(net, batch(777_777 + m, device, 32))))
        if before_step:
            before_step(gen, pop)
        pairs = pop.step(fitness)
        if after_step:
            after_step(gen, pop, pairs)
        best.append(max(fitness))
        log(f"generation {gen}: best fitness {best[-1]:.4f}, pairs {pairs}")
    return best


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--generations", type=int, default=4)
    ap.add_argument("--population", type=int, default=4)
    ap.add_argument("--inner-steps", type=int, default=10)
    ap.add_argument("--elitism", type=int, default=1)
    a = ap.parse_args()
    run(a.generations, a.population, a.inner_steps, a.elitism)


if __name__ == "__main__":
    main()
