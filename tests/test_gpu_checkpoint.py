"""The checkpoint write edge from a device arena (checkpoint.write_from_arena: pooled pinned staging
pair, D2H of chunk i+1 overlapping the write of chunk i) — the files the reference's
save_pretrained would leave (EDT_LM/diloco.py:302-308, EDT_EVOMERGE/train/crossover.py:140-146)."""
from __future__ import annotations

import pytest
import torch

from evolutionarydistributedtraining_amd import checkpoint
from evolutionarydistributedtraining_amd.params import ParamLayout

pytestmark = pytest.mark.gpu

SHAPES = [(1000, 37), (5,), (70001,), (3, 3), (1,), (4096, 33)]
NAMES = [f"layers.{i}.weight" for i in range(len(SHAPES))]


@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.skip("needs a HIP device")
    return torch.device("cuda:0")


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("staging", [4096, 1 << 20, 64 << 20])
def test_write_from_device_arena_streams_every_byte(tmp_path, dev, dtype, staging):
    from safetensors.torch import load_file
    layout = ParamLayout(SHAPES, NAMES)
    g = torch.Generator(device=dev).manual_seed(5)
    src = torch.randn(layout.total, device=dev, generator=g)
    flat = (src * 3).to(dtype)            # produced on the current stream just before the write
    path = str(tmp_path / "model.safetensors")
    checkpoint.write_from_arena(path, layout, flat, staging_bytes=staging)
    got = load_file(path)
    host = flat.cpu()
    assert sorted(got) == sorted(NAMES)
    for name, v in zip(NAMES, layout.views(host)):
        assert got[name].dtype == dtype
        assert torch.equal(got[name], v), name
    back = torch.empty_like(flat)
    checkpoint.read_into_arena(str(tmp_path), layout, back)
    torch.cuda.synchronize()
    assert torch.equal(back.cpu(), host)
    assert not (tmp_path / "model.safetensors.tmp").exists()


def test_write_from_device_arena_rejects_a_strided_view(tmp_path, dev):
    layout = ParamLayout([(8,)], ["w"])
    x = torch.zeros(16, device=dev)[::2]
    with pytest.raises(ValueError):
        checkpoint.write_from_arena(str(tmp_path / "m.safetensors"), layout, x)


@pytest.mark.parametrize("shard_bytes", [1 << 10, 300_000, 1 << 30])
def test_sharded_write_from_device_arena(tmp_path, dev, shard_bytes):
    """write_sharded_from_arena from a device arena just produced on the current stream: every
    shard streamed whole (one writer thread and staging pair per shard), the index names each
    tensor's shard, and the directory reads back into an arena bit for bit."""
    import json
    from safetensors.torch import load_file
    layout = ParamLayout(SHAPES, NAMES)
    g = torch.Generator(device=dev).manual_seed(7)
    flat = (torch.randn(layout.total, device=dev, generator=g) * 3).to(torch.bfloat16)
    files = checkpoint.write_sharded_from_arena(str(tmp_path), layout, flat, shard_bytes, staging_bytes=1 << 16)
    idx = json.load(open(tmp_path / "model.safetensors.index.json"))
    assert sorted(set(idx["weight_map"].values())) == sorted(files) and sorted(idx["weight_map"]) == sorted(NAMES)
    host = flat.cpu()
    for name, v in zip(NAMES, layout.views(host)):
        assert torch.equal(load_file(str(tmp_path / idx["weight_map"][name]))[name], v), name
    back = torch.empty_like(flat)
    checkpoint.read_into_arena(str(tmp_path), layout, back)
    torch.cuda.synchronize()
    assert torch.equal(back.cpu(), host)
    assert not any(p.name.endswith(".tmp") for p in tmp_path.iterdir())
