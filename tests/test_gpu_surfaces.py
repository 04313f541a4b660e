"""The reference's call surfaces, end to end on the GPU, against the golden vectors the reference
produced: DiLoCo `outer_step` on model parameter lists, the EDT-LM `run_sgd` / `crossover_main`
worker flow (HF folders, genome.json, outer_optim.pt), the RL `crossover(g1, g2, out)` over
Policy/Value folders and the EVOMERGE `run_slerp_merge_from_config` on bf16 Qwen2 bodies.
Tolerances as in test_gpu_kernels.py (SLERP: fp64 vs fp32 dot; bf16: scalar-tail rounding)."""
import json
import os

import numpy as np
import pytest
import torch
from safetensors.torch import load_file

from tests.golden_data import bits, flat

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    return torch.device("cuda:0")


def _ulp_bf16(x):
    a = x.float().abs().clamp_min(torch.finfo(torch.bfloat16).tiny)
    return torch.exp2(torch.floor(torch.log2(a)) - 7)


def _tiny_llama_cfg(dtype="bfloat16"):
    from transformers import LlamaConfig
    return LlamaConfig(vocab_size=24, hidden_size=8, intermediate_size=16, num_hidden_layers=4,
                       num_attention_heads=2, num_key_value_heads=1, tie_word_embeddings=False, dtype=dtype)


def _llama(tensors, dtype=torch.bfloat16, cfg_dtype="bfloat16"):
    from transformers import LlamaForCausalLM
    m = LlamaForCausalLM(_tiny_llama_cfg(cfg_dtype)).to(dtype)
    with torch.no_grad():
        for p, t in zip(m.parameters(), tensors):
            p.copy_(t)
    return m


def _save_tokenizer(path):
    from tokenizers import Tokenizer, models, pre_tokenizers
    from transformers import PreTrainedTokenizerFast
    vocab = {"[UNK]": 0, **{f"w{i}": i + 1 for i in range(23)}}
    tok = Tokenizer(models.WordLevel(vocab, unk_token="[UNK]"))
    tok.pre_tokenizer = pre_tokenizers.Whitespace()
    PreTrainedTokenizerFast(tokenizer_object=tok, unk_token="[UNK]").save_pretrained(path)


# ------------------------------------------------------------------------------------------
def test_diloco_outer_step_surface(golden, oracle, dev):
    """outer_step(list(base.parameters()), [list(m.parameters())...], state) over two generations,
    arena (flat launch) and separate-tensor (tensor-list launch) paths, vs the reference goldens."""
    from evolutionarydistributedtraining_amd import OuterState, arena_of_module, outer_step
    c = [c for c in golden.diloco_cases() if c["K"] == 3 and c["global_dtype"] == "f32"
         and c["worker_dtype"] == "f32" and c["nesterov"] and c["momentum"] == 0.9][0]
    T = len(c["shapes"])
    for zero_copy, placed in ((True, False), (False, False), (True, True)):
        # placed: OuterState(place_momentum=4) — the buffer's placement chosen by measurement when
        # the arena path creates it; values unchanged
        state = OuterState(place_momentum=4) if placed else None
        for step in c["steps"]:
            pre = step["prefix"]
            base = torch.nn.ParameterList([torch.nn.Parameter(t.clone()) for t in golden.tlist("diloco", f"{pre}/base", T)]).to(dev)
            trained = [torch.nn.ParameterList([torch.nn.Parameter(t.clone()) for t in
                                               golden.tlist("diloco", f"{pre}/worker{k}", T)]).to(dev)
                       for k in range(c["K"])]
            if zero_copy:
                arena_of_module(base)
                for m in trained:
                    arena_of_module(m)
            state = outer_step(list(base.parameters()), [list(m.parameters()) for m in trained], state,
                               lr=c["lr"], momentum=c["momentum"], nesterov=c["nesterov"])
            got = flat([p.detach().cpu() for p in base.parameters()])
            want = flat(golden.tlist("diloco", f"{pre}/out_theta", T))
            assert torch.equal(bits(got), bits(want)), (pre, zero_copy)
            assert torch.equal(bits(state.momentum.cpu()), bits(flat(golden.tlist("diloco", f"{pre}/out_buf", T))))
        assert isinstance(state, OuterState) and state.steps == 2
        if placed:
            assert state.placement is not None and state.placement["candidates"] >= 1, state.placement


def _pair_case(golden, name):
    c = [c for c in golden.pair_cases() if c["name"].endswith(name)][0]
    T = c["n_tensors"]
    g = lambda tag: golden.tlist("pair_merge", f"{c['name']}/{tag}", T)
    return c, g


@pytest.mark.parametrize("name", ["both_parent1_rule", "p2_only", "gen0_fresh", "gen0_sig_defaults"])
def test_lm_run_sgd_surface(golden, oracle, dev, tmp_path, name):
    from evolutionarydistributedtraining_amd import lm_crossover
    from tests.test_oracle_golden import pair_inputs
    c, g = _pair_case(golden, name)
    p1 = tmp_path / "m1" / c["generation"]
    p2 = tmp_path / "m2" / c["generation"]
    out = tmp_path / "child"
    for d in (p1, p2):
        d.mkdir(parents=True)

    def write_optim(path, bufs):
        ps = [torch.nn.Parameter(b.clone()) for b in bufs]
        o = torch.optim.SGD(ps, lr=0.7, momentum=0.9, nesterov=True)
        for p, b in zip(ps, bufs):
            o.state[p]["momentum_buffer"] = b.clone()
        torch.save(o.state_dict(), path)
    if c["parent1_optim"]:
        write_optim(p1 / "outer_optim.pt", g("buf1"))
    if c["parent2_optim"]:
        write_optim(p2 / "outer_optim.pt", g("buf2"))
    m1, m2 = _llama(g("m1")).to(dev), _llama(g("m2")).to(dev)
    base = _llama(g("merged_base")).to(dev)
    lm_crossover.run_sgd(m1, m2, base, str(out), str(p1), str(p2), lr=c["call_lr"],
                         momentum=c["call_momentum"], nesterov=c["call_nesterov"])
    got = flat([p.detach().cpu() for p in base.parameters()])
    p = pair_inputs(golden, c)
    ref = torch.empty_like(got)
    mom = None if p["mom"] is None else p["mom"].clone()
    oracle.pair_merge(p["b1"], p["b2"], p["m1"], p["m2"], ref, mom, p["has"], p["lr"], p["mu"], p["nesterov"])
    assert torch.equal(bits(got), bits(ref))                        # == vectorised reference semantics
    want = flat(g("out_theta"))
    tail = oracle.torch_cpu_tail_mask([int(torch.Size(s).numel()) for s in c["shapes"]])
    diff = bits(got) != bits(want)
    assert not (diff & (tail == 0)).any()
    sd = torch.load(out / "outer_optim.pt", weights_only=True)
    assert sd["param_groups"][0]["momentum"] == p["mu"]
    if c["has_out_buf"]:
        got_buf = flat([sd["state"][i]["momentum_buffer"] for i in range(c["n_tensors"])])
        assert torch.equal(bits(got_buf), bits(flat(g("out_buf"))))
    else:
        assert sd["state"] == {}
    assert (out / "model.safetensors").exists()


def test_lm_run_sgd_requires_parent_state(dev, tmp_path, golden):
    from evolutionarydistributedtraining_amd import lm_crossover
    c, g = _pair_case(golden, "p1_only")
    m = _llama(g("m1")).to(dev)
    with pytest.raises(NotImplementedError):
        lm_crossover.run_sgd(m, m, _llama(g("b1")).to(dev), str(tmp_path / "o"), str(tmp_path / "a" / "Gen0003"),
                             str(tmp_path / "b" / "Gen0003"), 0.7, 0.9, True)


@pytest.mark.parametrize("direct", [True, False])
def test_lm_crossover_main_cli_flow(golden, oracle, dev, tmp_path, direct):
    """Parent dirs with genome.json -> child dir: model, tokenizer, genome, outer_optim.pt,
    optimizer.pt carried from parent 1's trained dir (EDT_LM/train/crossover.py:240-315).
    direct: parents read straight into HBM arenas; else through from_pretrained."""
    from evolutionarydistributedtraining_amd import lm_crossover
    from tests.test_oracle_golden import pair_inputs
    c, g = _pair_case(golden, "both_parent1_rule")
    dirs = {}
    for tag in ("1", "2"):
        base_dir = tmp_path / f"m{tag}" / "Gen0003"
        mut_dir = tmp_path / f"m{tag}" / "Gen0003_mutation"
        _llama(g(f"b{tag}")).save_pretrained(base_dir)
        _llama(g(f"m{tag}")).save_pretrained(mut_dir)
        _save_tokenizer(mut_dir)
        (mut_dir / "optimizer.pt").write_bytes(f"inner-optimizer-{tag}".encode())
        ps = [torch.nn.Parameter(b.clone()) for b in g(f"buf{tag}")]
        o = torch.optim.SGD(ps, lr=0.7, momentum=0.9, nesterov=True)
        for p_, b in zip(ps, g(f"buf{tag}")):
            o.state[p_]["momentum_buffer"] = b.clone()
        torch.save(o.state_dict(), base_dir / "outer_optim.pt")
        with open(base_dir / "genome.json", "w") as f:
            json.dump({"fitness": 1.0, "model_path": str(base_dir), "mutation_path": str(mut_dir),
                       "dna": [0, 1, 2] if tag == "1" else [3, 2, 1], "p1": {"x": 1}}, f)
        dirs[tag] = base_dir
    out = tmp_path / "child" / "Gen0004"
    np.random.seed(123)
    lm_crossover.crossover_main(str(dirs["1"]), str(dirs["2"]), str(out), direct=direct)
    sd = load_file(str(out / "model.safetensors"))
    from transformers import LlamaForCausalLM
    names = [n for n, _ in LlamaForCausalLM(_tiny_llama_cfg()).named_parameters()]
    got = flat([sd[n] for n in names])
    p = pair_inputs(golden, c)
    ref = torch.empty_like(got)
    oracle.pair_merge(p["b1"], p["b2"], p["m1"], p["m2"], ref, p["mom"].clone(), True, 0.7, 0.9, True)
    assert torch.equal(bits(got), bits(ref))
    genome = json.load(open(out / "genome.json"))
    np.random.seed(123)
    from evolutionarydistributedtraining_amd.merge import uniform_dna_crossover
    assert genome["dna"] == uniform_dna_crossover([0, 1, 2], [3, 2, 1])
    assert "p1" not in genome["p1"] and genome["fitness"] == 0.0 and genome["model_path"] == str(out)
    assert (out / "optimizer.pt").read_bytes() == b"inner-optimizer-1"
    assert (out / "tokenizer.json").exists() or (out / "tokenizer_config.json").exists()
    osd = torch.load(out / "outer_optim.pt", weights_only=True)
    got_buf = flat([osd["state"][i]["momentum_buffer"] for i in range(c["n_tensors"])])
    assert torch.equal(bits(got_buf), bits(flat(g("out_buf"))))


def _slerp_tol(want_out, p1, p2, rel=3e-6):
    return rel * (p1.float().abs() + p2.float().abs()) + 1e-30


def test_rl_crossover_surface(golden, dev, tmp_path):
    """crossover(g1, g2, out) over Policy/Value folders (fp32), vs the reference's saved output."""
    from transformers import LlamaForCausalLM
    from evolutionarydistributedtraining_amd import rl_crossover
    t = golden.tensors("merge_models")
    rec = [r for r in golden.manifest["merge_models"] if r["name"] == "rl_crossover"][0]
    gs = {}
    for tag in ("p1", "p2"):
        root = tmp_path / tag
        for part in ("Policy", "Value"):
            m = LlamaForCausalLM(_tiny_llama_cfg("float32"))
            keys = rec["parts"][part]["keys"]
            sd = {"model." + k: t[f"merge_models/rl/{part}/{tag}/{k}"] for k in keys}
            sd["lm_head.weight"] = torch.zeros_like(m.lm_head.weight)
            m.load_state_dict(sd)
            m.save_pretrained(root / part)
        gs[tag] = {"model_path": str(root), "env": {"env_name": "wb",
                   "reward_dna": [1, 2, 3, 4, 5, 6] if tag == "p1" else [6, 5, 4, 3, 2, 1], "agents": []}}
    np.random.seed(rec["np_seed"])
    child = rl_crossover.crossover(gs["p1"], gs["p2"], str(tmp_path / "child"))
    assert child["env"]["reward_dna"] == rec["reward_dna"]
    assert child["p1"] is gs["p1"] and child["model_path"] == str(tmp_path / "child")
    for part in ("Policy", "Value"):
        out = load_file(str(tmp_path / "child" / part / "model.safetensors"))
        for k in rec["parts"][part]["keys"]:
            want = t[f"merge_models/rl/{part}/out/{k}"]
            a, b = t[f"merge_models/rl/{part}/p1/{k}"], t[f"merge_models/rl/{part}/p2/{k}"]
            assert out[k].dtype == torch.float32
            assert ((out[k] - want).abs() <= _slerp_tol(want, a, b)).all(), (part, k)


@pytest.mark.parametrize("ref", [False, True])
def test_evomerge_surface(golden, dev, tmp_path, ref):
    """run_slerp_merge_from_config on bf16 Qwen2 bodies, result written into model_1 (bf16): the
    single pass into a fresh buffer, model_1's parameters re-pointed at it (merge.slerp_into_module_).
    ref=True (merge.set_reference_dot(RefDot())): the reference's saved output, bit for bit."""
    from transformers import Qwen2Config, Qwen2ForCausalLM
    from evolutionarydistributedtraining_amd import evomerge_crossover as ev
    from evolutionarydistributedtraining_amd import merge, ops
    t = golden.tensors("merge_models")
    rec = [r for r in golden.manifest["merge_models"] if r["name"] == "evomerge"][0]
    cfg = Qwen2Config(vocab_size=24, hidden_size=8, intermediate_size=16, num_hidden_layers=5,
                      num_attention_heads=2, num_key_value_heads=1, tie_word_embeddings=False)
    models = []
    for tag in ("p1", "p2"):
        m = Qwen2ForCausalLM(cfg).to(torch.bfloat16)
        m.model.load_state_dict({k: t[f"merge_models/evomerge/{tag}/{k}"] for k in rec["keys"]})
        with torch.no_grad():
            m.lm_head.weight.copy_(t["merge_models/evomerge/out_lm_head"])
        models.append(m.to(dev))
    merge_cfg = ev.slerp_config("a", "b", 5)
    before = {k: p.data_ptr() for k, p in models[0].model.named_parameters()}
    prev = merge.set_reference_dot(ops.RefDot() if ref else None)
    try:
        ev.run_slerp_merge_from_config(merge_cfg, models[0].model, models[1].model, cfg, cfg, str(tmp_path / "o"),
                                       base_model=models[0])
    finally:
        merge.set_reference_dot(prev)
    after = {k: p.data_ptr() for k, p in models[0].model.named_parameters()}
    assert all(after[k] != before[k] for k in rec["keys"])          # re-pointed at the fresh buffer
    sd = models[0].model.state_dict()
    n_exact = n = 0
    for k in rec["keys"]:
        want = t[f"merge_models/evomerge/out/{k}"]
        got = sd[k].cpu()
        assert got.dtype == torch.bfloat16
        if ref:
            assert torch.equal(got.view(torch.int16), want.view(torch.int16)), k
        d = (got.float() - want.float()).abs()
        assert (d <= _ulp_bf16(want) * 1.0001).all(), k          # fp32 result within tol -> <= 1 bf16 ulp
        n_exact += int((d == 0).sum())
        n += d.numel()
    assert n_exact / n > 0.98
    assert torch.equal(models[0].lm_head.weight.cpu(), t["merge_models/evomerge/out_lm_head"])
    assert (tmp_path / "o" / "model.safetensors").exists()


def test_single_tensor_slerp_api(golden, dev):
    """slerp(t, v0, v1) on CPU tensors / numpy arrays / device tensors returns like the reference."""
    from evolutionarydistributedtraining_amd.merge import slerp
    ts = golden.tensors("slerp")
    c = [c for c in golden.slerp_cases() if c["name"] == "slerp/generic_f32_t2"][0]
    v0, v1 = ts[f"{c['inputs']}/v0"], ts[f"{c['inputs']}/v1"]
    want = ts[f"{c['name']}/out"]
    r_cpu = slerp(c["t"], v0, v1)
    assert r_cpu.device.type == "cpu" and r_cpu.shape == want.shape
    assert ((r_cpu - want).abs() <= _slerp_tol(want, v0, v1)).all()
    r_np = slerp(c["t"], v0.numpy(), v1.numpy())
    assert isinstance(r_np, np.ndarray)
    r_dev = slerp(c["t"], v0.to(dev), v1.to(dev))
    assert r_dev.is_cuda and torch.equal(r_dev.cpu(), r_cpu)


def test_dir_outer_sync_two_generations(oracle, dev, tmp_path):
    """DirOuterSync with its DEFAULT arguments (so the one-time momentum placement search of
    place_momentum=8 runs after the first step): checkpoint dirs in, fused step, checkpoint dirs out
    (EDT_LM/diloco.py:224-308), two generations with the momentum carried across a master restart
    (state_path), bit-identical to the oracle — theta every generation, the momentum at the end;
    outputs load with HF."""
    from transformers import LlamaForCausalLM
    from evolutionarydistributedtraining_amd.diloco import DirOuterSync
    from evolutionarydistributedtraining_amd.params import ParamLayout, pack
    K = 3
    base = _llama([p.detach() for p in _llama([]).parameters()], torch.bfloat16)
    g = torch.Generator().manual_seed(21)
    with torch.no_grad():
        for p in base.parameters():
            p.copy_(torch.randn(p.shape, generator=g) * 0.02)
    layout = ParamLayout.of_module(base)
    base.save_pretrained(tmp_path / "w0" / "Gen0000")
    state_path = str(tmp_path / "outer_optim.pt")
    sync = DirOuterSync(device=dev, names=layout.names, lr=0.7, momentum=0.9, nesterov=True, state_path=state_path)
    theta = pack(list(base.parameters()))
    mom = torch.zeros_like(theta)
    prev = str(tmp_path / "w0" / "Gen0000")
    for gen in range(2):
        dirs = []
        workers = []
        for k in range(K):
            d = tmp_path / f"w{k}" / f"Gen{gen + 1:04d}"
            m = _llama([(t.float() + torch.randn(t.shape, generator=g) * 1e-3).bfloat16()
                        for t in layout.views(theta)])
            m.save_pretrained(d)
            dirs.append(str(d))
            workers.append(pack(list(m.parameters())))
        if gen == 1:        # a restarted master: the momentum carry comes back from state_path
            sync = DirOuterSync(device=dev, names=layout.names, lr=0.7, momentum=0.9, nesterov=True,
                                state_path=state_path)
        sync.step(prev, dirs)
        assert sync.placement is not None          # the default search ran (and moved nothing's values)
        oracle.outer_step(theta, workers, mom, gen > 0, 0.7, 0.9, True)
        for d in dirs:
            got = LlamaForCausalLM.from_pretrained(d, dtype=torch.bfloat16)
            assert torch.equal(bits(pack(list(got.parameters()))), bits(theta)), (gen, d)
        prev = dirs[0]
    assert torch.equal(bits(sync.state.momentum.cpu()), bits(mom))


def test_dir_outer_sync_placed_momentum_and_inner_state_carry(oracle, dev, tmp_path):
    """DirOuterSync(place_momentum=8, carry_inner_state=True): the whole resident set (θ, worker
    arenas, momentum) placed once after the first step (placement.place_set; resident arenas, so
    the placement holds), every later generation bit-identical to
    the oracle; each GenN+1 dir ends with its machine's GenN optimizer.pt / scheduler.pt
    (EDT_LM/diloco.py:295-300)."""
    from transformers import LlamaForCausalLM
    from evolutionarydistributedtraining_amd.diloco import DirOuterSync
    from evolutionarydistributedtraining_amd.params import ParamLayout, pack
    K = 2
    base = _llama([p.detach() for p in _llama([]).parameters()], torch.bfloat16)
    g = torch.Generator().manual_seed(22)
    with torch.no_grad():
        for p in base.parameters():
            p.copy_(torch.randn(p.shape, generator=g) * 0.02)
    layout = ParamLayout.of_module(base)
    for k in range(K):
        base.save_pretrained(tmp_path / f"w{k}" / "Gen0000")
        (tmp_path / f"w{k}" / "Gen0000" / "optimizer.pt").write_bytes(f"opt w{k} g0".encode())
        (tmp_path / f"w{k}" / "Gen0000" / "scheduler.pt").write_bytes(f"sch w{k} g0".encode())
    sync = DirOuterSync(device=dev, names=layout.names, lr=0.7, momentum=0.9, nesterov=True,
                        carry_inner_state=True, place_momentum=8, place_draws=3)
    theta = pack(list(base.parameters()))
    mom = torch.zeros_like(theta)
    prev = [str(tmp_path / f"w{k}" / "Gen0000") for k in range(K)]
    for gen in range(3):
        dirs, workers = [], []
        for k in range(K):
            d = tmp_path / f"w{k}" / f"Gen{gen + 1:04d}"
            m = _llama([(t.float() + torch.randn(t.shape, generator=g) * 1e-3).bfloat16()
                        for t in layout.views(theta)])
            m.save_pretrained(d)
            (d / "optimizer.pt").write_bytes(f"opt w{k} g{gen + 1}".encode())
            dirs.append(str(d))
            workers.append(pack(list(m.parameters())))
        sync.step(prev[0], dirs, prev_dirs=prev)
        oracle.outer_step(theta, workers, mom, gen > 0, 0.7, 0.9, True)
        for k, d in enumerate(dirs):
            got = LlamaForCausalLM.from_pretrained(d, dtype=torch.bfloat16)
            assert torch.equal(bits(pack(list(got.parameters()))), bits(theta)), (gen, d)
            assert (tmp_path / f"w{k}" / f"Gen{gen + 1:04d}" / "optimizer.pt").read_bytes() == f"opt w{k} g0".encode()
        assert sync.placement is not None and sync.placement["candidates"] >= 1
        assert len(sync.placement["draws"]) >= 1 and sync.placement["chosen_draw"] is not None
        prev = dirs
    assert torch.equal(bits(sync.state.momentum.cpu()), bits(mom))


@pytest.mark.parametrize("wdt", [torch.bfloat16, torch.float32])
@pytest.mark.parametrize("mode,broadcast", [("reduce", "theta"), ("exact", "theta"), ("exact", "workers")])
def test_sharded_outer_step_rccl_world1(oracle, dev, tmp_path, mode, broadcast, wdt):
    """The multi-GPU schedule on the real RCCL backend (one rank: the collectives degenerate, but
    the in-place reduce-scatter / all-gather, async waits and stream ordering are RCCL's)."""
    import torch.distributed as dist
    from evolutionarydistributedtraining_amd.distributed import ShardedOuterSync
    from evolutionarydistributedtraining_amd.params import ParamLayout
    store = dist.FileStore(str(tmp_path / "store"), 1)
    dist.init_process_group("nccl", store=store, rank=0, world_size=1, device_id=dev)
    try:
        layout = ParamLayout([(1000, 37), (4097,), (3,)])
        sync = ShardedOuterSync(layout, torch.float32, wdt, 3, dev, 0.7, 0.9, True, mode=mode,
                                bucket_elems=8192, broadcast=broadcast)
        assert (sync.mode, sync.broadcast) == (mode, broadcast) and len(sync.buckets) > 3
        g = torch.Generator().manual_seed(8)
        theta = torch.randn(layout.total, generator=g) * 0.02
        mom = torch.zeros(layout.total)
        sync.theta.flat.copy_(theta)
        for step in range(2):
            ws = [(theta + torch.randn(layout.total, generator=g) * 1e-3).to(wdt) for _ in range(3)]
            for a, w in zip(sync.workers, ws):
                a.flat.copy_(w)
            sync.step()
            oracle.outer_step(theta, ws, mom, step > 0, 0.7, 0.9, True)
        torch.cuda.synchronize()
        if broadcast == "workers":
            for a in sync.workers:
                assert torch.equal(bits(a.flat.cpu()), bits(theta.to(wdt)))
        assert torch.equal(bits(sync.gather_theta().cpu()), bits(theta))   # fp32: same order, bit-exact
        assert torch.equal(bits(sync.mom_shard[:layout.total].cpu()), bits(mom))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("tdt", [torch.float32, torch.bfloat16])
def test_momentum_placement_keeps_the_step_bit_identical(dev, tdt):
    """OuterSync.place_momentum moves the momentum to the fastest of several allocations
    (placement.py); contents and every later step stay bit-identical, exact zeros in theta
    included (the probe kernel it times rewrites theta and momentum)."""
    from evolutionarydistributedtraining_amd.diloco import OuterSync
    from evolutionarydistributedtraining_amd.params import ParamArena, ParamLayout
    layout = ParamLayout([torch.Size((1000, 1000)), torch.Size((4097,)), torch.Size((3,))], ["a", "b", "c"])
    g = torch.Generator(device=dev).manual_seed(11)
    theta0 = (torch.randn(layout.total, generator=g, device=dev) * 0.02).to(tdt)
    theta0[:5000] = 0                                     # exact zeros must survive the probe
    ws0 = [(theta0.float() + torch.randn(layout.total, generator=g, device=dev) * 1e-3).to(tdt)
           for _ in range(3)]
    syncs = []
    for place in (False, True):
        theta = ParamArena(layout, tdt, dev)
        theta.flat.copy_(theta0)
        workers = [ParamArena(layout, tdt, dev) for _ in ws0]
        for w, w0 in zip(workers, ws0):
            w.flat.copy_(w0)
        s = OuterSync(theta, workers, 0.7, 0.9, True)
        s.step()
        if place:
            before_t, before_m = theta.flat.clone(), s.state.momentum.clone()
            rep = s.place_momentum(3)
            assert rep["candidates"] == 3 and len(rep["probe_ms"]) == 3 and 0 <= rep["chosen"] < 3
            assert torch.equal(theta.flat, before_t) and torch.equal(s.state.momentum, before_m)
        s.step()
        s.step()
        syncs.append(s)
    a, b = syncs
    assert torch.equal(a.theta.flat.view(torch.int16 if tdt == torch.bfloat16 else torch.int32),
                       b.theta.flat.view(torch.int16 if tdt == torch.bfloat16 else torch.int32))
    assert torch.equal(a.state.momentum, b.state.momentum)


@pytest.mark.parametrize("tdt", [torch.float32, torch.bfloat16])
def test_arena_placement_keeps_the_step_bit_identical(dev, tdt):
    """OuterSync.place_arenas (r6) draws the whole operand set — theta, the workers, the momentum —
    in several regions of HBM and keeps the fastest: the arenas are re-pointed with their contents
    unchanged (exact zeros included), and every later step is bit-identical to the unplaced run."""
    from evolutionarydistributedtraining_amd.diloco import OuterSync
    from evolutionarydistributedtraining_amd.params import ParamArena, ParamLayout
    layout = ParamLayout([torch.Size((1000, 1000)), torch.Size((4097,)), torch.Size((3,))], ["a", "b", "c"])
    g = torch.Generator(device=dev).manual_seed(12)
    theta0 = (torch.randn(layout.total, generator=g, device=dev) * 0.02).to(tdt)
    theta0[:5000] = 0
    ws0 = [(theta0.float() + torch.randn(layout.total, generator=g, device=dev) * 1e-3).to(tdt) for _ in range(3)]
    syncs = []
    for place in (False, True):
        theta = ParamArena(layout, tdt, dev)
        theta.flat.copy_(theta0)
        workers = [ParamArena(layout, tdt, dev) for _ in ws0]
        for w, w0 in zip(workers, ws0):
            w.flat.copy_(w0)
        s = OuterSync(theta, workers, 0.7, 0.9, True)
        s.step()
        if place:
            before = [theta.flat.clone(), s.state.momentum.clone()] + [w.flat.clone() for w in workers]
            rep = s.place_arenas(draws=3, candidates=3)
            assert len(rep["draws"]) == 3 and 0 <= rep["chosen_draw"] < 3, rep
            assert rep["momentum"]["candidates"] == 3
            after = [theta.flat, s.state.momentum] + [w.flat for w in workers]
            assert all(torch.equal(x, y) for x, y in zip(before, after))
        s.step()
        s.step()
        syncs.append(s)
    a, b = syncs
    vb = torch.int16 if tdt == torch.bfloat16 else torch.int32
    assert torch.equal(a.theta.flat.view(vb), b.theta.flat.view(vb))
    assert torch.equal(a.state.momentum.view(vb), b.state.momentum.view(vb))
    for wa, wb in zip(a.workers, b.workers):
        assert torch.equal(wa.flat.view(vb), wb.flat.view(vb))


def test_place_set_one_draw_and_the_memory_limit(dev):
    """place_set with one draw is the momentum search on the set where it lies (theta and the
    workers returned as they were); a draw that does not fit free memory is not taken — the report
    names it (draws_limited_by_memory) and the first draw's set comes back."""
    from evolutionarydistributedtraining_amd.placement import place_set
    n = 1 << 20
    g = torch.Generator(device=dev).manual_seed(3)
    theta = torch.randn(n, generator=g, device=dev)
    workers = [theta + torch.randn(n, generator=g, device=dev) * 1e-3 for _ in range(2)]
    mom = torch.randn(n, generator=g, device=dev) * 1e-3
    keep = [theta.clone(), mom.clone()] + [w.clone() for w in workers]
    th, ws, m, rep = place_set(theta, workers, mom, draws=1, candidates=3)
    assert th is theta and all(a is b for a, b in zip(ws, workers))
    assert len(rep["draws"]) == 1 and rep["chosen_draw"] == 0 and rep["candidates"] == 3
    assert "draws_limited_by_memory" not in rep
    assert all(torch.equal(x, y) for x, y in zip(keep, [th, m] + ws))
    free, _ = torch.cuda.mem_get_info(dev)
    th, ws, m, rep = place_set(theta, workers, m, draws=3, candidates=2, spacer_bytes=free)
    assert rep["draws_limited_by_memory"] == 1 and rep["chosen_draw"] == 0 and len(rep["draws"]) == 1
    assert th is theta and all(a is b for a, b in zip(ws, workers))
    assert all(torch.equal(x, y) for x, y in zip(keep, [th, m] + ws))


# ------------------------------------------------------------------------------------------
# libedt_comm.so (include/edt_comm.h) at world size 1 on the one-GPU box: the collectives are
# identities, the sharded reduce schedule equals the single-GPU fused step bit for bit (fp32 master)

def test_comm_abi_world1_collectives(dev):
    from evolutionarydistributedtraining_amd.comm import Comm
    c = Comm(Comm.unique_id(), 1, 0)
    try:
        assert (c.rank, c.size) == (0, 1)
        g = torch.Generator(device=dev).manual_seed(5)
        x = torch.randn(4099, generator=g, device=dev)
        y = torch.empty_like(x)
        c.reduce_scatter_f32(x, y)
        torch.cuda.synchronize()
        assert torch.equal(x, y)
        for dt in (torch.float32, torch.bfloat16):
            xs, ys = x.to(dt), torch.empty(4099, dtype=dt, device=dev)
            c.all_gather(xs, ys)
            torch.cuda.synchronize()
            assert torch.equal(xs, ys)
            ys.zero_()
            c.all_to_all(xs, ys)
            torch.cuda.synchronize()
            assert torch.equal(xs, ys)
        a, b = torch.arange(1000, dtype=torch.int32, device=dev), torch.zeros(1000, dtype=torch.int32, device=dev)
        c.exchange([(0, a, 0, b)])                 # a grouped send to self and receive from self
        torch.cuda.synchronize()
        assert torch.equal(a, b)
    finally:
        c.close()


@pytest.mark.parametrize("wdt", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("schedule", ["reduce", "ordered", "exact"])
def test_comm_abi_sharded_outer_step_world1(dev, wdt, schedule):
    """edt_outer_step_sharded (reduce), edt_outer_step_sharded_ordered (reduce_ordered: the
    partials' all-to-all + edt_sgd_apply_sum) and edt_outer_step_sharded_exact (the workers'
    all-to-all + the fused step per shard) at world 1: bit-exact with the fused step over the
    whole population, over several buckets and a padded tail."""
    from evolutionarydistributedtraining_amd import ops
    from evolutionarydistributedtraining_amd.comm import Comm
    n, n_pad, K = 100_003, 100_032, 5                      # n_pad: a multiple of 64 (world 1)
    g = torch.Generator(device=dev).manual_seed(9)
    theta0 = torch.zeros(n_pad, device=dev)
    theta0[:n] = torch.randn(n, generator=g, device=dev) * 0.02
    workers = []
    for _ in range(K):
        w = torch.zeros(n_pad, dtype=wdt, device=dev)
        w[:n] = (theta0[:n] + torch.randn(n, generator=g, device=dev) * 1e-3).to(wdt)
        workers.append(w)
    ref_t, ref_m = theta0.clone(), torch.zeros(n_pad, device=dev)
    th, mom, acc = theta0.clone(), torch.zeros(n_pad, device=dev), torch.empty(n_pad, device=dev)
    recv = torch.empty(n_pad, device=dev)
    recv_w = [torch.empty(n_pad, dtype=wdt, device=dev) for _ in range(K)]
    c = Comm(Comm.unique_id(), 1, 0)
    try:
        for has in (False, True, True):
            ops.outer_step(ref_t, workers, ref_m, has, 0.7, 0.9, True)
            if schedule == "ordered":
                c.outer_step_sharded_ordered(th, workers, mom, has, 0.7, 0.9, True, acc, recv, bucket_elems=16_384)
            elif schedule == "exact":
                c.outer_step_sharded_exact(th, workers, mom, has, 0.7, 0.9, True, recv_w, bucket_elems=16_384)
            else:
                c.outer_step_sharded(th, workers, mom, has, 0.7, 0.9, True, acc, bucket_elems=16_384)
        torch.cuda.synchronize()
    finally:
        c.close()
    assert torch.equal(th.view(torch.int32), ref_t.view(torch.int32))
    assert torch.equal(mom.view(torch.int32), ref_m.view(torch.int32))
    assert not th[n:].any()


def test_comm_abi_bounded_step_and_abort_world1(dev):
    """The failure path of include/edt_comm.h: with a timeout set, the sharded step waits for its
    work (polling RCCL's async error) and returns done; after edt_comm_abort every call fails
    with a negative code and a message (EDT_COMM_ERR_ABORTED), and the handle still closes."""
    from evolutionarydistributedtraining_amd import _lib as L
    from evolutionarydistributedtraining_amd.comm import ERR_ABORTED, Comm, load_comm_library
    n = 64 * 1000
    g = torch.Generator(device=dev).manual_seed(2)
    th = torch.randn(n, generator=g, device=dev) * 0.02
    ws = [th + torch.randn(n, generator=g, device=dev) * 1e-3 for _ in range(3)]
    mom, acc = torch.zeros(n, device=dev), torch.empty(n, device=dev)
    c = Comm(Comm.unique_id(), 1, 0)
    try:
        c.poll()
        c.set_timeout(60.0)
        ref = th.clone()
        ops_mom = torch.zeros(n, device=dev)
        from evolutionarydistributedtraining_amd import ops
        ops.outer_step(ref, ws, ops_mom, False, 0.7, 0.9, True)
        c.outer_step_sharded(th, ws, mom, False, 0.7, 0.9, True, acc, bucket_elems=8192)
        c.wait(dev, timeout_s=60.0)
        assert torch.equal(th.view(torch.int32), ref.view(torch.int32))
        c.abort()
        lib = load_comm_library()
        rc = lib.edt_comm_reduce_scatter_f32(c._h, L.ptr(acc), L.ptr(acc), n, L.stream_ptr(dev))
        assert rc == ERR_ABORTED and b"aborted" in lib.edt_comm_last_error()
        with pytest.raises(L.EdtError, match="aborted"):
            c.poll()
        with pytest.raises(L.EdtError, match="aborted"):
            c.outer_step_sharded(th, ws, mom, True, 0.7, 0.9, True, acc, bucket_elems=8192)
        with pytest.raises(L.EdtError, match="aborted"):
            c.wait(dev, timeout_s=1.0)
    finally:
        c.close()


def test_outer_step_surface_cpu_tails_bit_exact_with_reference(golden, dev):
    """diloco.outer_step(..., cpu_tails=(32, threads)) on the golden case generated with torch's
    parallel chunks (separate parameter tensors, as list(model.parameters())): the reference's
    bf16 output and momentum, bit for bit."""
    from evolutionarydistributedtraining_amd.diloco import outer_step
    from tests.golden_data import bits, flat
    c = golden.manifest["diloco_large"]
    T = len(c["shapes"])
    pre = c["name"]
    base = [t.clone().to(dev) for t in golden.tlist("diloco", f"{pre}/s0/base", T)]
    state = None
    for step in (0, 1):
        ws = [[t.to(dev) for t in golden.tlist("diloco", f"{pre}/s{step}/worker{k}", T)] for k in range(c["K"])]
        state = outer_step(base, ws, state, c["lr"], c["momentum"], c["nesterov"],
                           cpu_tails=(32, c["torch_num_threads"]))
        got = flat([t.cpu() for t in base])
        assert torch.equal(bits(got), bits(flat(golden.tlist("diloco", f"{pre}/s{step}/out_theta", T)))), step


def _qwen_pair(dev, far, seed=0):
    from transformers import Qwen2Config, Qwen2ForCausalLM
    cfg = Qwen2Config(vocab_size=40, hidden_size=32, intermediate_size=72, num_hidden_layers=4,
                      num_attention_heads=4, num_key_value_heads=2, tie_word_embeddings=False)
    g = torch.Generator().manual_seed(seed)
    ms = [Qwen2ForCausalLM(cfg).to(torch.bfloat16) for _ in range(2)]
    with torch.no_grad():
        for p1, p2 in zip(ms[0].parameters(), ms[1].parameters()):
            p1.copy_(torch.randn(p1.shape, generator=g) * 0.02)
            noise = torch.randn(p1.shape, generator=g) * 0.02
            p2.copy_(noise if far else p1.float() + noise * 0.005)
    return cfg, [m.to(dev) for m in ms]


@pytest.mark.parametrize("far", [False, True])
def test_evomerge_rebind_equals_in_place(dev, far):
    """merge_models_into_(model_1, model_1, model_2) — the single pass into a fresh buffer, then
    model_1's parameters re-pointed — gives the bits of the in-place two-pass merge into model_1's
    own tensors, leaves model_2 alone, and a second generation on the re-pointed parameters too."""
    from evolutionarydistributedtraining_amd import evomerge_crossover as ev
    from evolutionarydistributedtraining_amd import merge
    cfg, (m1, m2) = _qwen_pair(dev, far)
    mcfg = ev.slerp_config("a", "b", cfg.num_hidden_layers)
    start = {k: v.clone() for k, v in m1.model.state_dict().items()}
    m2_bits = {k: v.clone() for k, v in m2.model.state_dict().items()}
    plan = merge.merge_plan(list(start), cfg.num_hidden_layers, mcfg)
    for gen in range(2):
        want_sd = {k: v.clone() for k, v in m1.model.state_dict().items()}
        merge.slerp_state_dicts(dict(want_sd), m2.model.state_dict(), plan, out_dtype=torch.bfloat16,
                                device=dev, out=want_sd)                      # in place, two-pass
        before = {k: p.data_ptr() for k, p in m1.model.named_parameters()}
        merge.merge_models_into_(m1.model, m1.model, m2.model, mcfg, cfg.num_hidden_layers, device=dev)
        got = m1.model.state_dict()
        for k, _ in plan:
            assert got[k].data_ptr() != before[k]
            assert got[k].dtype == torch.bfloat16 and got[k].is_contiguous()
            assert torch.equal(got[k].view(torch.int16), want_sd[k].view(torch.int16)), (gen, k)
        assert all(torch.equal(v, m2_bits[k]) for k, v in m2.model.state_dict().items())


def test_evomerge_mixed_dtype_target_keeps_its_tensors(dev):
    """A bf16 model_1 with one fp32 parameter: not re-pointed (a fresh bf16 buffer would change that
    parameter's dtype); the merge is written into model_1's tensors in their own dtypes, as
    load_state_dict does, each tensor equal to its own single-tensor merge."""
    from evolutionarydistributedtraining_amd import evomerge_crossover as ev
    from evolutionarydistributedtraining_amd import merge
    cfg, (m1, m2) = _qwen_pair(dev, far=True, seed=1)
    with torch.no_grad():
        m1.model.norm.weight.data = m1.model.norm.weight.data.float()
    mcfg = ev.slerp_config("a", "b", cfg.num_hidden_layers)
    sd1 = {k: v.clone() for k, v in m1.model.state_dict().items()}
    sd2 = m2.model.state_dict()
    plan = merge.merge_plan(list(sd1), cfg.num_hidden_layers, mcfg)
    before = {k: (p.data_ptr(), p.dtype) for k, p in m1.model.named_parameters()}
    merge.merge_models_into_(m1.model, m1.model, m2.model, mcfg, cfg.num_hidden_layers, device=dev)
    got = m1.model.state_dict()
    for k, t in plan:
        assert (got[k].data_ptr(), got[k].dtype) == before[k], k
        want = merge.slerp_tensors([(sd1[k], sd2[k])], [t], out_dtype=torch.float32, device=dev)[0]
        assert torch.equal(got[k], want.to(got[k].dtype)), k


def test_evomerge_repeat_binding_follows_module_changes(dev, monkeypatch):
    """merge_models_into_'s cached binding (merge._Bound, VERDICT r4 Next 3): the repeat of a merge
    into model_1 launches over the cached addresses and checks the modules while the device runs.
    Every generation equals the in-place two-pass merge bit for bit, whatever changed in between:
    nothing (the cached launch), model_1 written in place (same addresses: cached), a model_2
    parameter re-pointed, a model_1 Parameter replaced by a new one (both: the check fails, the
    uncached merge runs, the new binding is recorded), every model_1 tensor re-pointed (caught before
    the launch: no cached launch is spent); the entry dies with model_2."""
    import gc

    from evolutionarydistributedtraining_amd import evomerge_crossover as ev
    from evolutionarydistributedtraining_amd import merge
    merge.clear_merge_cache()
    cfg, (m1, m2) = _qwen_pair(dev, far=False, seed=7)
    mcfg = ev.slerp_config("a", "b", cfg.num_hidden_layers)
    plan = merge.merge_plan(list(m1.model.state_dict()), cfg.num_hidden_layers, mcfg)
    hits = []
    real = merge._bound_merge
    monkeypatch.setattr(merge, "_bound_merge", lambda b, x, y: hits.append(real(b, x, y)) or hits[-1])
    cached_launches = []
    real_checked = merge.ops.SlerpListBinding.from_checked
    monkeypatch.setattr(merge.ops.SlerpListBinding, "from_checked",
                        lambda *a, **k: cached_launches.append(1) or real_checked(*a, **k))

    def change(gen):
        with torch.no_grad():
            if gen == 2:
                m1.model.layers[0].mlp.up_proj.weight.mul_(1.5)               # in place: same addresses
            elif gen == 3:
                w = m2.model.layers[1].self_attn.q_proj.weight
                w.data = w.data.clone() * 0.5                                # model_2 re-pointed
            elif gen == 4:
                lin = m1.model.layers[2].self_attn.o_proj
                lin.weight = torch.nn.Parameter(lin.weight.detach().clone())  # a new Parameter
            elif gen == 6:
                for p in m1.model.parameters():                               # a reload: all moved
                    p.data = p.data.clone()

    expect = [None, True, True, False, False, True, False, True]
    for gen in range(8):
        change(gen)
        want = {k: v.clone() for k, v in m1.model.state_dict().items()}
        merge.slerp_state_dicts(dict(want), m2.model.state_dict(), plan, out_dtype=torch.bfloat16, device=dev,
                                out=want)
        n, c = len(hits), len(cached_launches)
        merge.merge_models_into_(m1.model, m1.model, m2.model, mcfg, cfg.num_hidden_layers, device=dev)
        assert (hits[n] if len(hits) > n else None) == expect[gen], (gen, hits)
        if gen == 6:
            assert len(cached_launches) == c, "a moved model_1 must be caught before the cached launch"
        got = m1.model.state_dict()
        for k, _ in plan:
            assert torch.equal(got[k].view(torch.int16), want[k].view(torch.int16)), (gen, k)
    assert len(merge._bound_cache) == 1
    del m2
    gc.collect()
    assert len(merge._bound_cache) == 0
