"""Checkpoint edge: HF save_pretrained directories (single file and sharded) read straight into a
flat parameter arena, and arenas written back as safetensors that HF loads unchanged. I/O only,
so the arena may live on the CPU here; the GPU form is exercised in scripts/e2e_rate.py."""
import os
import shutil

import pytest
import torch
from safetensors.torch import load_file

from evolutionarydistributedtraining_amd import checkpoint
from evolutionarydistributedtraining_amd.params import ParamArena, ParamLayout, pack


def _tiny(dtype):
    from transformers import LlamaConfig, LlamaForCausalLM
    cfg = LlamaConfig(vocab_size=40, hidden_size=16, intermediate_size=24, num_hidden_layers=3,
                      num_attention_heads=2, num_key_value_heads=1, tie_word_embeddings=False)
    torch.manual_seed(0)
    return LlamaForCausalLM(cfg).to(dtype)


@pytest.mark.parametrize("shard", [None, "8KB"])
@pytest.mark.parametrize("ckpt_dtype,arena_dtype", [(torch.bfloat16, torch.bfloat16), (torch.float32, torch.float32),
                                                    (torch.bfloat16, torch.float32)])
def test_read_hf_checkpoint_into_arena(tmp_path, shard, ckpt_dtype, arena_dtype):
    m = _tiny(ckpt_dtype)
    kw = {"max_shard_size": shard} if shard else {}
    m.save_pretrained(tmp_path, **kw)
    if shard:
        assert os.path.exists(tmp_path / "model.safetensors.index.json")
    layout = ParamLayout.of_module(m)
    arena = ParamArena(layout, arena_dtype, "cpu")
    checkpoint.read_into_arena(str(tmp_path), layout, arena.flat, staging_bytes=4096)
    want = pack(list(m.parameters()), dtype=arena_dtype)
    assert torch.equal(arena.flat, want)


def test_write_arena_is_loadable_by_safetensors_and_hf(tmp_path):
    from transformers import LlamaForCausalLM
    m = _tiny(torch.bfloat16)
    m.save_pretrained(tmp_path / "src")
    layout = ParamLayout.of_module(m)
    flat = pack(list(m.parameters())) * 2
    out = tmp_path / "dst"
    checkpoint.save_to_dirs([str(out), str(tmp_path / "dst2")], layout, flat)
    sd = load_file(str(out / "model.safetensors"))
    for (name, p), v in zip(m.named_parameters(), layout.views(flat)):
        assert torch.equal(sd[name], v)
    shutil.copy(tmp_path / "src" / "config.json", out / "config.json")
    m2 = LlamaForCausalLM.from_pretrained(out, dtype=torch.bfloat16)
    for a, b in zip(m2.parameters(), layout.views(flat)):
        assert torch.equal(a, b)
    assert (tmp_path / "dst2" / "model.safetensors").read_bytes() == (out / "model.safetensors").read_bytes()


def test_shape_mismatch_is_an_error(tmp_path):
    m = _tiny(torch.float32)
    m.save_pretrained(tmp_path)
    layout = ParamLayout.of_module(m)
    bad = ParamLayout([(1,)] + layout.shapes[1:], layout.names)
    with pytest.raises(ValueError):
        checkpoint.read_into_arena(str(tmp_path), bad, torch.empty(bad.total))


def test_read_many_parallel_matches_serial(tmp_path):
    """checkpoint.read_many (one reader thread per checkpoint, pooled staging) fills every arena
    exactly as read_into_arena does one after another."""
    layout = None
    dirs, want = [], []
    for k in range(5):
        m = _tiny(torch.bfloat16)
        with torch.no_grad():
            for p in m.parameters():
                p.add_(k)                       # distinct checkpoints
        d = tmp_path / f"w{k}"
        m.save_pretrained(d, **({"max_shard_size": "8KB"} if k % 2 else {}))
        layout = layout or ParamLayout.of_module(m)
        dirs.append(str(d))
        want.append(pack(list(m.parameters())))
    arenas = [torch.full((layout.total,), float("nan"), dtype=torch.bfloat16) for _ in dirs]
    checkpoint.read_many(list(zip(dirs, arenas)), layout, threads=4, staging_bytes=4096)
    for a, w in zip(arenas, want):
        assert torch.equal(a, w)


def test_broadcast_copies_are_independent_files(tmp_path):
    """save_to_dirs gives every worker dir its own file with the same bytes (no hard links), so a
    worker rewriting its checkpoint in place (save_pretrained truncates; EDT_LM/diloco.py:302-308's
    next generation) leaves the others intact, and no temporary file is left behind."""
    m = _tiny(torch.float32)
    layout = ParamLayout.of_module(m)
    flat = pack(list(m.parameters()))
    dirs = [str(tmp_path / f"w{k}") for k in range(4)]
    checkpoint.save_to_dirs(dirs, layout, flat)
    files = [os.path.join(d, "model.safetensors") for d in dirs]
    ref = open(files[0], "rb").read()
    assert len({os.stat(f).st_ino for f in files}) == 4
    assert all(open(f, "rb").read() == ref for f in files)
    with open(files[1], "wb") as f:                   # an in-place rewrite of one worker's file
        f.write(b"x")
    assert all(open(f, "rb").read() == ref for f in files[:1] + files[2:])
    assert not any(n.endswith(".tmp") for d in dirs for n in os.listdir(d))
    sd = load_file(files[3])
    for (name, _), v in zip(m.named_parameters(), layout.views(flat)):
        assert torch.equal(sd[name], v)


def test_broadcast_over_existing_files_unlinks_then_renames(tmp_path):
    """The broadcast lands over the workers' trained checkpoints (the outer step's out_dirs are its
    worker dirs): each old file is renamed away before the complete new one is renamed into place
    (checkpoint._publish: no rename replaces a file, so ext4 does not flush the new file
    synchronously) and deleted in the background. The path ends with the new bytes on a new inode;
    another name of the old file keeps the old bytes; once flush_deletions returns nothing but the
    new files is left; an old name left by a dead process is deleted by the next publish there;
    copy_file unlinks an existing target for the carried inner-state files."""
    m = _tiny(torch.float32)
    layout = ParamLayout.of_module(m)
    flat = pack(list(m.parameters()))
    dirs = [str(tmp_path / f"w{k}") for k in range(3)]
    for d in dirs:
        os.makedirs(d)
        with open(os.path.join(d, "model.safetensors"), "wb") as f:
            f.write(b"trained replica")
    keep = str(tmp_path / "old_link")
    os.link(os.path.join(dirs[0], "model.safetensors"), keep)
    old_ino = os.stat(keep).st_ino
    dead = os.path.join(dirs[1], "model.safetensors" + checkpoint._TRASH + "999999999-0")
    open(dead, "wb").write(b"left by a dead process")
    checkpoint.save_to_dirs(dirs, layout, flat)
    checkpoint.flush_deletions()
    assert sorted(os.listdir(dirs[1])) == ["model.safetensors"] and os.listdir(dirs[2]) == ["model.safetensors"]
    files = [os.path.join(d, "model.safetensors") for d in dirs]
    ref = open(files[0], "rb").read()
    assert ref != b"trained replica" and all(open(f, "rb").read() == ref for f in files)
    assert os.stat(files[0]).st_ino != old_ino and open(keep, "rb").read() == b"trained replica"
    assert not any(n.endswith(".tmp") for d in dirs for n in os.listdir(d))
    src, dst = str(tmp_path / "opt_src.pt"), os.path.join(dirs[1], "optimizer.pt")
    open(src, "wb").write(b"carried")
    open(dst, "wb").write(b"trained")
    os.link(dst, str(tmp_path / "opt_link"))
    checkpoint.copy_file(src, dst)
    assert open(dst, "rb").read() == b"carried" and open(str(tmp_path / "opt_link"), "rb").read() == b"trained"
    checkpoint.copy_file(src, os.path.join(dirs[2], "optimizer.pt"))     # no file there yet
    assert open(os.path.join(dirs[2], "optimizer.pt"), "rb").read() == b"carried"


def test_broadcast_over_a_sharded_replica_reads_back_the_broadcast(tmp_path):
    """A worker dir holding its trained replica as index + shards (a model too big for one
    file) receives the new global model from save_to_dirs (EDT_LM/diloco.py:302-308): the stale
    index and shards are removed, and reading the dir back (a restarted master, _read_parents_direct)
    returns the broadcast weights, not the trained ones."""
    m = _tiny(torch.float32)
    d = tmp_path / "w0"
    m.save_pretrained(d, max_shard_size="8KB")
    assert os.path.exists(d / "model.safetensors.index.json")
    layout = ParamLayout.of_module(m)
    new = pack(list(m.parameters())) * 3 + 1
    checkpoint.save_to_dirs([str(d)], layout, new)
    left = sorted(os.listdir(d))
    assert "model.safetensors.index.json" not in left
    assert not any(f.startswith("model-") for f in left)
    got = checkpoint.read_into_arena(str(d), layout, torch.empty(layout.total))
    assert torch.equal(got, new)


def test_single_file_wins_over_a_stale_index(tmp_path):
    """checkpoint_files resolves model.safetensors before an index, as transformers does."""
    m = _tiny(torch.float32)
    d = tmp_path / "w"
    m.save_pretrained(d, max_shard_size="8KB")
    layout = ParamLayout.of_module(m)
    new = pack(list(m.parameters())) - 5
    checkpoint.write_from_arena(str(d / "model.safetensors"), layout, new)
    assert os.path.exists(d / "model.safetensors.index.json")
    assert set(checkpoint.checkpoint_files(str(d)).values()) == {str(d / "model.safetensors")}
    got = checkpoint.read_into_arena(str(d), layout, torch.empty(layout.total))
    assert torch.equal(got, new)


def test_split_readers_and_threaded_writes(tmp_path):
    """read_many with fewer checkpoints than readers cuts each checkpoint into tensor ranges (one
    reader each); the threaded pwrite writer produces the same file as a single write."""
    m = _tiny(torch.bfloat16)
    m.save_pretrained(tmp_path / "a", max_shard_size="8KB")
    layout = ParamLayout.of_module(m)
    want = pack(list(m.parameters()))
    got = torch.full((layout.total,), float("nan"), dtype=torch.bfloat16)
    checkpoint.read_many([(str(tmp_path / "a"), got)], layout, threads=5, staging_bytes=4096)
    assert torch.equal(got, want)
    header = checkpoint._header_bytes(layout, layout.names, want.dtype, None)
    checkpoint._write_file(str(tmp_path / "one.safetensors"), header, want, threads=1)
    checkpoint._write_file(str(tmp_path / "many.safetensors"), header, want, threads=7, min_bytes=0)
    assert (tmp_path / "one.safetensors").read_bytes() == (tmp_path / "many.safetensors").read_bytes()
    sd = load_file(str(tmp_path / "many.safetensors"))
    for (name, _), v in zip(m.named_parameters(), layout.views(want)):
        assert torch.equal(sd[name], v)


from hypothesis import HealthCheck, given, settings  # noqa: E402
from hypothesis import strategies as st  # noqa: E402


def _write_sharded(d, names, tensors, cuts):
    """A HF-style sharded checkpoint written by hand: files split at `cuts` (tensor indices),
    tensors stored in a shuffled order inside each file, plus model.safetensors.index.json."""
    import json
    import random

    from safetensors.torch import save_file
    os.makedirs(d, exist_ok=True)
    bounds = [0] + sorted(set(cuts)) + [len(names)]
    nf = len(bounds) - 1
    wmap = {}
    rng = random.Random(len(names) * 7 + nf)
    for f in range(nf):
        idx = list(range(bounds[f], bounds[f + 1]))
        rng.shuffle(idx)
        fname = f"model-{f + 1:05d}-of-{nf:05d}.safetensors"
        save_file({names[i]: tensors[i].contiguous() for i in idx}, os.path.join(d, fname))
        for i in idx:
            wmap[names[i]] = fname
    with open(os.path.join(d, "model.safetensors.index.json"), "w") as fh:
        json.dump({"metadata": {}, "weight_map": wmap}, fh)


@settings(max_examples=40, deadline=None, derandomize=True,
          suppress_health_check=[HealthCheck.function_scoped_fixture, HealthCheck.too_slow])
@given(shapes=st.lists(st.one_of(st.tuples(st.integers(1, 5000)), st.tuples(st.integers(1, 60), st.integers(1, 60))),
                       min_size=1, max_size=9),
       ckpt_dt=st.sampled_from([torch.float32, torch.bfloat16]), arena_dt=st.sampled_from([torch.float32, torch.bfloat16]),
       cuts=st.lists(st.integers(1, 8), max_size=3), staging=st.sampled_from([64, 4096, 1 << 20]),
       threads=st.integers(1, 8), copies=st.integers(1, 3), seed=st.integers(0, 2**31 - 1))
def test_reader_fuzz(tmp_path_factory, shapes, ckpt_dt, arena_dt, cuts, staging, threads, copies, seed):
    """read_into_arena / read_many over random layouts, shard splits, in-file tensor orders, dtype
    conversions (torch copy_ rounding, as load_state_dict does), staging sizes smaller than one
    tensor, and reader counts (one checkpoint split over several readers): every arena equals the
    tensors packed in layout order."""
    d0 = str(tmp_path_factory.mktemp("ck"))
    g = torch.Generator().manual_seed(seed)
    names = [f"layers.{i}.w" for i in range(len(shapes))]
    layout = ParamLayout([torch.Size(s) for s in shapes], names)
    items, want = [], []
    for c in range(copies):
        ts = [(torch.randn(s, generator=g) * 0.02).to(ckpt_dt) for s in shapes]
        d = os.path.join(d0, f"m{c}")
        _write_sharded(d, names, ts, [k for k in cuts if k < len(shapes)])
        items.append((d, torch.full((layout.total,), float("nan"), dtype=arena_dt)))
        want.append(torch.cat([t.reshape(-1).to(arena_dt) for t in ts]))
    checkpoint.read_many(items, layout, threads=threads, staging_bytes=staging)
    for (_, flat), w in zip(items, want):
        assert torch.equal(flat, w)


def test_sharded_write_reads_back_and_loads_in_hf(tmp_path):
    """write_sharded_from_arena: HF's sharded layout (shards of whole tensors <= shard_bytes +
    index) that read_into_arena and from_pretrained both load; a single-file save there before is
    removed, and rewriting with another shard count leaves no stale shard behind."""
    from transformers import LlamaForCausalLM
    m = _tiny(torch.bfloat16)
    m.save_pretrained(tmp_path / "src")
    layout = ParamLayout.of_module(m)
    flat = pack(list(m.parameters())) * 3
    d = tmp_path / "child"
    checkpoint.save_to_dirs([str(d)], layout, flat * 0)             # a single-file save first
    files = checkpoint.write_sharded_from_arena(str(d), layout, flat, shard_bytes=4096)
    assert len(files) > 2 and not (d / "model.safetensors").exists()
    assert sorted(os.listdir(d)) == sorted(files + ["model.safetensors.index.json"])
    back = torch.empty_like(flat)
    checkpoint.read_into_arena(str(d), layout, back)
    assert torch.equal(back, flat)
    shutil.copy(tmp_path / "src" / "config.json", d / "config.json")
    m2 = LlamaForCausalLM.from_pretrained(d, dtype=torch.bfloat16)
    for a, b in zip(m2.parameters(), layout.views(flat)):
        assert torch.equal(a, b)
    few = checkpoint.write_sharded_from_arena(str(d), layout, flat + 1, shard_bytes=1 << 20)
    assert len(few) == 1 and sorted(f for f in os.listdir(d) if f.endswith(".safetensors")) == few
    checkpoint.read_into_arena(str(d), layout, back)
    assert torch.equal(back, flat + 1)
