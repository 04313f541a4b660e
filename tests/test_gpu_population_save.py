"""ResidentPopulation.save / load with the members on the device and the HIP kernels: the files are
written by several writer threads at once (one per checkpoint, r6), each ordered after the caller's
current stream — here a side stream that produced the last generation — and a fresh population
load()ed from them holds every arena bit for bit."""
import random

import numpy as np
import pytest
import torch

from tests.test_population import SHAPES, _fitness, _genomes, _init, _noise

pytestmark = pytest.mark.gpu


def test_resident_population_save_load_on_device(tmp_path):
    from evolutionarydistributedtraining_amd.params import ParamLayout
    from evolutionarydistributedtraining_amd.population import ResidentPopulation
    dev = torch.device("cuda:0")
    layout = ParamLayout(SHAPES)
    n, dt = layout.total, torch.bfloat16
    random.seed(3)
    np.random.seed(3)
    a = ResidentPopulation(layout, dt, dev, _genomes("sgd"), elitism=1)
    side = torch.cuda.Stream(dev)
    with torch.cuda.stream(side):
        for m in a.local_members():
            a.base(m).copy_(_init(m, n, dt).to(dev))
        for gen in range(2):
            a.begin_inner()
            for m in a.local_members():
                t = a.trained(m)
                t.copy_((t.float() + _noise(gen, m, n).to(dev)).to(dt))
            a.step(_fitness(gen))
        a.save(str(tmp_path / "ckpt"))             # on the side stream that produced the arenas
    torch.cuda.synchronize()
    b = ResidentPopulation(layout, dt, dev, _genomes("sgd"), elitism=1)
    b.load(str(tmp_path / "ckpt"))
    torch.cuda.synchronize()
    assert b.generation == a.generation and b.genomes == a.genomes
    for m in a.local_members():
        assert torch.equal(b.base(m).view(torch.int16), a.base(m).view(torch.int16)), m
        ma, mb = a.outer_momentum(m), b.outer_momentum(m)
        assert (ma is None) == (mb is None), m
        if ma is not None:
            assert torch.equal(mb.view(torch.int16), ma.view(torch.int16)), m
    assert any(a.outer_momentum(m) is not None for m in a.local_members())
