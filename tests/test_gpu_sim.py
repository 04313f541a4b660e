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
