"""DirOuterSync over checkpoint directories on the CPU (the fused kernel swapped for the oracle's
outer step, which is bit-exact with it; the GPU form is tests/test_gpu_surfaces.py): the file layout
EDT_LM/diloco.py:291-308 leaves behind, including the inner-state carry of :295-300 —

    for source, target in zip(prev_gen_dirs, curr_gen_dirs):      # GenN -> GenN+1 of each machine
        copy source/{optimizer.pt, scheduler.pt} over target's, where the source file exists
    then the outer-stepped base model is saved to every GenN+1 dir.

Restated here as the expected layout: each GenN+1 dir ends with the new weights, its machine's GenN
optimizer.pt / scheduler.pt (or its own when GenN had none), and the base's config."""
import json
import os

import pytest
import torch
from safetensors.torch import load_file, save_file

SHAPES = {"embed.weight": (40, 16), "layer.0.weight": (16, 16), "layer.0.bias": (16,), "head.weight": (40, 16)}


def _write_model(d, tensors, extra=None):
    os.makedirs(d, exist_ok=True)
    save_file(tensors, os.path.join(d, "model.safetensors"))
    with open(os.path.join(d, "config.json"), "w") as f:
        json.dump({"model_type": "tiny", "hidden_size": 16}, f)
    for name, payload in (extra or {}).items():
        with open(os.path.join(d, name), "wb") as f:
            f.write(payload)


def _layout(root, K, gen, seed, with_prev_state):
    """machine{i}/Gen{gen} (the base, identical on every machine) and machine{i}/Gen{gen+1} (the
    trained replica with the inner loop's own optimizer.pt / scheduler.pt)."""
    g = torch.Generator().manual_seed(seed)
    base = {k: torch.randn(s, generator=g) * 0.02 for k, s in SHAPES.items()}
    prev, curr = [], []
    for i in range(K):
        p = os.path.join(root, f"machine{i}", f"Gen{gen:04d}")
        c = os.path.join(root, f"machine{i}", f"Gen{gen + 1:04d}")
        state = {"optimizer.pt": f"inner-opt m{i} g{gen}".encode(), "scheduler.pt": f"sched m{i} g{gen}".encode()}
        if not with_prev_state[i]:
            state = {}
        _write_model(p, base, state)
        trained = {k: v + torch.randn(v.shape, generator=g) * 1e-3 for k, v in base.items()}
        _write_model(c, trained, {"optimizer.pt": f"inner-opt m{i} g{gen + 1}".encode(),
                                  "scheduler.pt": f"sched m{i} g{gen + 1}".encode(), "trainer_state.json": b"{}"})
        prev.append(p)
        curr.append(c)
    return base, prev, curr


def _oracle_sync(monkeypatch, oracle):
    from evolutionarydistributedtraining_amd import diloco

    def outer_step(theta, workers, mom, has, lr, mu, nesterov, broadcast=None, tail_bits=None):
        oracle.outer_step(theta, workers, mom, has, lr, mu, nesterov)
        for b in broadcast or []:
            b.copy_(theta)

    monkeypatch.setattr(diloco.ops, "outer_step", outer_step)
    return diloco


@pytest.mark.parametrize("carry", [True, False])
def test_dir_outer_sync_file_layout(tmp_path, monkeypatch, oracle, carry):
    diloco = _oracle_sync(monkeypatch, oracle)
    K = 3
    names = list(SHAPES)
    with_prev = [True, False, True]          # machine 1's GenN has no inner state: its own stays
    base, prev, curr = _layout(str(tmp_path), K, 0, 1, with_prev)
    before = {c: {f: open(os.path.join(c, f), "rb").read() for f in ("optimizer.pt", "scheduler.pt")} for c in curr}
    trained = [load_file(os.path.join(c, "model.safetensors")) for c in curr]
    sync = diloco.DirOuterSync(device="cpu", names=names, lr=0.7, momentum=0.9, nesterov=True,
                               carry_inner_state=carry)
    sync.step(prev[0], curr, prev_dirs=prev if carry else None)
    # expected: the oracle's outer step over the flat parameters in `names` order
    flat = lambda ts: torch.cat([ts[n].reshape(-1) for n in names])   # noqa: E731
    theta = flat(base).clone()
    oracle.outer_step(theta, [flat(t) for t in trained], torch.zeros_like(theta), False, 0.7, 0.9, True)
    for i, c in enumerate(curr):
        got = load_file(os.path.join(c, "model.safetensors"))
        assert torch.equal(flat(got), theta), c
        for f in ("optimizer.pt", "scheduler.pt"):
            data = open(os.path.join(c, f), "rb").read()
            if carry and with_prev[i]:
                assert data == open(os.path.join(prev[i], f), "rb").read(), (c, f)
            else:
                assert data == before[c][f], (c, f)
        assert os.path.exists(os.path.join(c, "config.json"))
        assert open(os.path.join(c, "trainer_state.json"), "rb").read() == b"{}"   # untouched


def test_dir_outer_sync_carry_needs_prev_dirs(tmp_path, monkeypatch, oracle):
    diloco = _oracle_sync(monkeypatch, oracle)
    base, prev, curr = _layout(str(tmp_path), 2, 0, 2, [True, True])
    sync = diloco.DirOuterSync(device="cpu", names=list(SHAPES), carry_inner_state=True)
    with pytest.raises(ValueError):
        sync.step(prev[0], curr)
    with pytest.raises(ValueError):
        sync.step(prev[0], curr, prev_dirs=prev[:1])


def test_dir_outer_sync_two_generations_carry_momentum_and_state(tmp_path, monkeypatch, oracle):
    """Gen0 -> Gen1 -> Gen2 as the reference's master loop runs it: theta stays resident, the
    momentum is carried in RAM, and each generation's inner state is carried from the previous."""
    diloco = _oracle_sync(monkeypatch, oracle)
    names = list(SHAPES)
    K = 2
    root = str(tmp_path)
    base, prev, curr = _layout(root, K, 0, 3, [True, True])
    sync = diloco.DirOuterSync(device="cpu", names=names, carry_inner_state=True)
    sync.step(prev[0], curr, prev_dirs=prev)
    # inner loops of generation 1: new trained replicas in Gen0002, each with its own inner state
    g = torch.Generator().manual_seed(9)
    nxt = []
    for i in range(K):
        src = load_file(os.path.join(curr[i], "model.safetensors"))
        d = os.path.join(root, f"machine{i}", "Gen0002")
        _write_model(d, {k: v + torch.randn(v.shape, generator=g) * 1e-3 for k, v in src.items()},
                     {"optimizer.pt": f"inner-opt m{i} g2".encode(), "scheduler.pt": b"s2"})
        nxt.append(d)
    sync.step(curr[0], nxt, prev_dirs=curr)
    for i in range(K):
        assert open(os.path.join(nxt[i], "optimizer.pt"), "rb").read() == open(os.path.join(prev[i], "optimizer.pt"), "rb").read()
    assert sync.state.has_momentum and sync.state.steps == 2


def test_dir_outer_sync_carry_goes_beside_the_weights(tmp_path, monkeypatch, oracle):
    """out_dirs apart from worker_dirs: the carried inner state lands where the new
    weights are written, so the next inner loop finds both together; worker_dirs keep their own."""
    diloco = _oracle_sync(monkeypatch, oracle)
    base, prev, curr = _layout(str(tmp_path), 2, 0, 4, [True, True])
    outs = [os.path.join(str(tmp_path), f"out{i}") for i in range(2)]
    before = [open(os.path.join(c, "optimizer.pt"), "rb").read() for c in curr]
    sync = diloco.DirOuterSync(device="cpu", names=list(SHAPES), carry_inner_state=True)
    sync.step(prev[0], curr, out_dirs=outs, prev_dirs=prev)
    for i in range(2):
        assert os.path.exists(os.path.join(outs[i], "model.safetensors"))
        for f in ("optimizer.pt", "scheduler.pt"):
            assert open(os.path.join(outs[i], f), "rb").read() == open(os.path.join(prev[i], f), "rb").read()
        assert open(os.path.join(curr[i], "optimizer.pt"), "rb").read() == before[i]
