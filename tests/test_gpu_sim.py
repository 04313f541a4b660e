"""End-to-end DiLoCo simulation (examples/diloco_sim.py, the shape of the reference's
EDT_LM/diloco_sim.py — its only integration test): K workers train copies of a tiny
transformer LM on one GPU, the package's outer step merges them, generation after generation.
Every generation's outer step is checked against the reference's own loop restated
(oracle.torch_loop_outer_step: per tensor, the running sum of (trained - base) / K, grad = -sum,
torch.optim.SGD carried across generations) on CPU copies: bit-exact in fp32."""
import os
import sys

import pytest
import torch

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.skip("needs a HIP device")
    return torch.device("cuda:0")


def test_diloco_sim_outer_steps_match_the_reference_loop(oracle, dev):
    sys.path.insert(0, os.path.join(ROOT, "examples"))
    import diloco_sim
    ref = {"base": None, "opt": None}
    checked = []

    def before(gen, base, replicas):
        # the reference master's view: the global model and the K trained replicas, on its CPU
        if ref["base"] is None:
            ref["base"] = [p.detach().cpu().clone() for p in base.parameters()]
        else:       # the reference carries its own global model across generations
            for r, p in zip(ref["base"], base.parameters()):
                assert torch.equal(r.detach(), p.detach().cpu())
        ref["workers"] = [[p.detach().cpu().clone() for p in m.parameters()] for m in replicas]

    def after(gen, base, state):
        ref["opt"] = oracle.torch_loop_outer_step(ref["base"], ref["workers"], ref["opt"], 0.7, 0.9, True)
        for r, p in zip(ref["base"], base.parameters()):
            assert torch.equal(r.detach().view(torch.int32), p.detach().cpu().view(torch.int32)), gen
        checked.append(gen)

    evals = diloco_sim.run(generations=4, workers=3, inner_steps=8, device=dev, before_outer=before,
                           after_outer=after, log=lambda *_: None)
    assert checked == [0, 1, 2, 3]
    assert evals[-1] < evals[0]          # the outer loop learns the synthetic rule


def test_edt_sim_children_match_the_oracle(oracle, dev):
    """examples/edt_sim.py (the shape of EDT_LM/edt_sim.py): a resident population of tiny LMs
    trains, is scored and crossed generation after generation; every child (base and outer
    momentum) equals the oracle's pair merge of its parents' bases and trained weights with the
    donor's momentum (EDT_LM/train/crossover.py:150-237), bit for bit in fp32."""
    sys.path.insert(0, os.path.join(ROOT, "examples"))
    import edt_sim
    snap = {}
    checked = []

    def before(gen, pop):
        P = pop.P
        snap["base"] = [pop.base(m).cpu().clone() for m in range(P)]
        snap["trained"] = [pop.trained(m).cpu().clone() for m in range(P)]
        snap["mom"] = [pop.outer_momentum(m).cpu().clone() for m in range(P)]
        snap["has"] = list(pop.has_momentum)

    def after(gen, pop, pairs):
        for c, (i, j) in enumerate(pairs):
            donor = i if snap["has"][i] else (j if snap["has"][j] else None)
            n = snap["base"][0].numel()
            m_out = snap["mom"][donor].clone() if donor is not None else torch.zeros(n)
            out = torch.empty(n)
            oracle.pair_merge(snap["base"][i], snap["base"][j], snap["trained"][i], snap["trained"][j], out, m_out,
                              donor is not None, 0.7, 0.9, True)
            assert torch.equal(pop.base(c).cpu().view(torch.int32), out.view(torch.int32)), (gen, c)
            assert torch.equal(pop.outer_momentum(c).cpu().view(torch.int32), m_out.view(torch.int32)), (gen, c)
        checked.append(gen)

    best = edt_sim.run(generations=3, population=4, inner_steps=6, elitism=1, device=dev, before_step=before,
                       after_step=after, log=lambda *_: None)
    assert checked == [0, 1, 2]
    assert len(best) == 3
