"""Host-side logic of the shim (no GPU): key routing, t curves, DNA crossover, outer-state I/O,
parameter arenas, layouts, and the C ABI library surface."""
import os
import re

import numpy as np
import pytest
import torch

from evolutionarydistributedtraining_amd import merge
from evolutionarydistributedtraining_amd.diloco import OuterState
from evolutionarydistributedtraining_amd.layouts import LAYOUTS
from evolutionarydistributedtraining_amd.params import (ParamArena, ParamLayout, arena_of_module, flat_view,
                                                        pack, unpack_)

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_interpolate_t_matches_reference_tables(golden):
    for tab in golden.manifest["interpolate_t"]:
        got = [merge.interpolate_t(i, tab["num_layers"], tab["t_curve"]) for i in tab["layer_idx"]]
        assert got == tab["t"], tab          # python floats, bit-identical


def test_known_t_values():
    attn, mlp = [0, 0.5, 0.3, 0.7, 1], [1, 0.5, 0.7, 0.3, 0]
    assert [merge.interpolate_t(i, 4, attn) for i in range(4)] == pytest.approx([0, 0.43333, 0.56667, 1], abs=1e-5)
    assert [merge.interpolate_t(i, 4, mlp) for i in range(4)] == pytest.approx([1, 0.56667, 0.43333, 0], abs=1e-5)


def test_key_routing():
    cfg = {"parameters": {"t": [{"filter": "self_attn", "value": [0, 0.5, 0.3, 0.7, 1]},
                                {"filter": "mlp", "value": [1, 0.5, 0.7, 0.3, 0]}, {"value": 0.5}]}}
    param_t, global_t = merge.parse_t_parameters(cfg)
    assert global_t == 0.5 and set(param_t) == {"self_attn", "mlp"}
    assert merge.t_for_key("embed_tokens.weight", 4, param_t, global_t) == 0.5
    assert merge.t_for_key("norm.weight", 4, param_t, global_t) == 0.5
    assert merge.t_for_key("layers.0.self_attn.q_proj.weight", 4, param_t, global_t) == 0
    assert merge.t_for_key("layers.3.mlp.down_proj.weight", 4, param_t, global_t) == 0
    assert merge.t_for_key("layers.1.input_layernorm.weight", 4, param_t, global_t) == 0.5
    assert merge.t_for_key("layers.4.mlp.up_proj.weight", 4, param_t, global_t) is None      # skipped
    with pytest.raises(ValueError):                 # same failure as the reference's int() parse
        merge.t_for_key("model.layers.0.mlp.up_proj.weight", 4, param_t, global_t)
    # no global entry -> 0.5 default
    assert merge.parse_t_parameters({"parameters": {"t": [{"filter": "mlp", "value": [0, 1]}]}})[1] == 0.5


def test_merge_plan_on_golden_model_keys(golden):
    for case in golden.manifest["merge_models"]:
        if case["name"] != "evomerge":
            continue
        cfg = {"parameters": {"t": [{"filter": "self_attn", "value": [0, 0.5, 0.3, 0.7, 1]},
                                    {"filter": "mlp", "value": [1, 0.5, 0.7, 0.3, 0]}, {"value": 0.5}]}}
        plan = merge.merge_plan(case["keys"], case["num_hidden_layers"], cfg)
        assert [k for k, _ in plan] == case["keys"]


def test_uniform_dna_crossover_matches_reference_draws(golden):
    for rec in golden.manifest["dna_crossover"]:
        np.random.seed(rec["seed"])
        got = [merge.uniform_dna_crossover(rec["dna1"], rec["dna2"]) for _ in rec["draws"]]
        assert got == rec["draws"]
    with pytest.raises(AssertionError):
        merge.uniform_dna_crossover([1, 2], [1])


def test_python_number_lerp():
    assert merge.lerp(0.25, 1.0, 3.0) == (1 - 0.25) * 1.0 + 0.25 * 3.0


def test_outer_state_round_trip(tmp_path):
    layout = ParamLayout([(3, 2), (5,), (1,)])
    st = OuterState()
    st.momentum = torch.arange(layout.total, dtype=torch.float32)
    st.has_momentum = True
    st.hparams = dict(lr=0.7, momentum=0.9, nesterov=True)
    path = str(tmp_path / "outer_optim.pt")
    st.save(path, layout)
    sd = torch.load(path, weights_only=True)
    ref = torch.optim.SGD([torch.nn.Parameter(torch.zeros(1))], lr=0.7, momentum=0.9, nesterov=True).state_dict()
    assert set(sd["param_groups"][0]) == set(ref["param_groups"][0])
    assert sd["param_groups"][0]["params"] == [0, 1, 2]
    assert sd["state"][1]["momentum_buffer"].shape == (5,)
    st2 = OuterState.load(path, layout, torch.bfloat16, "cpu")
    assert st2.has_momentum and st2.momentum.dtype == torch.bfloat16
    assert torch.equal(st2.momentum.float(), st.momentum.bfloat16().float())
    # no buffers (momentum 0) -> fresh state
    st3 = OuterState()
    st3.hparams = dict(lr=1.0, momentum=0.0, nesterov=False)
    st3.save(path, layout)
    assert OuterState.load(path, layout, torch.float32, "cpu").momentum is None


def test_param_layout_and_views():
    ts = [torch.randn(3, 4), torch.randn(7), torch.randn(2, 2, 2)]
    flat = pack(ts)
    layout = ParamLayout.of(ts)
    assert layout.total == 12 + 7 + 8 and layout.offsets == [0, 12, 19, 27]
    views = layout.views(flat)
    assert all(torch.equal(a, b) for a, b in zip(views, ts))
    fv = flat_view(views)
    assert fv is not None and fv.data_ptr() == flat.data_ptr() and fv.numel() == flat.numel()
    assert flat_view(ts) is None                       # separate allocations
    assert flat_view([views[0], views[2]]) is None     # not consecutive
    for t in ts:
        t.zero_()
    unpack_(flat, ts)
    assert torch.equal(pack(ts), flat)


def test_bind_module_into_arena():
    m = torch.nn.Sequential(torch.nn.Linear(4, 3), torch.nn.Linear(3, 2))
    before = [p.detach().clone() for p in m.parameters()]
    arena = arena_of_module(m)
    assert all(torch.equal(a, b) for a, b in zip(m.parameters(), before))
    fv = flat_view(list(m.parameters()))
    assert fv is not None and fv.data_ptr() == arena.flat.data_ptr()
    arena.flat.add_(1.0)                                # an arena update is a module update
    assert all(torch.equal(a, b + 1) for a, b in zip(m.parameters(), before))
    assert isinstance(ParamArena.from_tensors(before), ParamArena)


@pytest.mark.parametrize("name,P,T", [("tiny_llama", 6_570_560, 39), ("gpt2_small", 124_439_808, 148),
                                      ("gpt_1p3b", 1_315_723_264, 292), ("qwen2p5_7b_body", 7_070_619_136, 338)])
def test_layouts_match_survey_counts(name, P, T):
    lay = LAYOUTS[name]()
    assert lay.total == P and len(lay) == T


def test_library_exports_every_header_symbol():
    from evolutionarydistributedtraining_amd import _lib
    lib = _lib.load_library()
    with open(os.path.join(ROOT, "include", "edt_sync.h")) as f:
        header = f.read()
    names = set(re.findall(r"^\s*(?:int|int64_t|uint64_t|const char\*)\s+(edt_\w+)\s*\(", header, re.M))
    assert len(names) >= 12
    for n in names:
        assert hasattr(lib, n), n
    bound = {n for n, _, _ in _lib.SIGNATURES}
    assert names == bound, names ^ bound
    assert lib.edt_version().startswith(b"edt_sync")
    assert lib.edt_outer_step_bytes_per_elem(0, 1, 8, 1) == 32


def test_comm_library_exports_every_header_symbol():
    """libedt_comm.so (include/edt_comm.h: RCCL behind the C ABI) loads without a GPU and binds
    every declared entry point; running them is the GPU tests' job."""
    from evolutionarydistributedtraining_amd import comm
    lib = comm.load_comm_library()
    with open(os.path.join(ROOT, "include", "edt_comm.h")) as f:
        header = f.read()
    names = set(re.findall(r"^\s*(?:int|uint64_t|const char\*)\s+(edt_\w+)\s*\(", header, re.M))
    assert len(names) == 18, names
    assert names == {n for n, _, _ in comm.SIGNATURES}
    for n in names:
        assert hasattr(lib, n), n
    assert lib.edt_comm_id_bytes() == 128


def test_c_consumer_builds_and_links():
    """tests/c_abi/abi_consumer.c includes only include/edt_sync.h (+ the HIP runtime) and links
    against libedt_sync.so with gcc: the boundary is usable with no Python in between. Running it
    needs a GPU (test_gpu_kernels.py::test_c_consumer_runs)."""
    import subprocess
    d = os.path.join(ROOT, "tests", "c_abi")
    subprocess.run(["make", "-s", "-C", d], check=True)
    out = subprocess.run(["ldd", os.path.join(d, "_build", "abi_consumer")], capture_output=True, text=True,
                         check=True, cwd="/").stdout
    assert "not found" not in out, out
    assert "libedt_sync.so" in out and "libamdhip64" in out
    # the plain-C multi-GPU master (include/edt_comm.h): libedt_comm.so and RCCL behind it
    out = subprocess.run(["ldd", os.path.join(d, "_build", "comm_consumer")], capture_output=True, text=True,
                         check=True, cwd="/").stdout
    assert "not found" not in out, out
    assert "libedt_comm.so" in out and "librccl" in out


def test_chunk_table_host_function():
    import ctypes
    from evolutionarydistributedtraining_amd import _lib
    lib = _lib.load_library()
    offs = (ctypes.c_uint64 * 5)(0, 0, 5, 70000, 70001)
    first = (ctypes.c_int32 * 5)()
    need = lib.edt_slerp_make_chunks(offs, 4, 32768, None, 0, first)
    assert need < 0
    n = -need - 1
    desc = (ctypes.c_uint64 * (3 * n))()
    assert lib.edt_slerp_make_chunks(offs, 4, 32768, desc, n, first) == n
    chunks = [tuple(desc[3 * i:3 * i + 3]) for i in range(n)]
    assert chunks == [(0, 5, 1), (5, 32768, 2), (32773, 32768, 2), (65541, 4459, 2), (70000, 1, 3)]
    assert list(first) == [0, 0, 1, 4, 5]


def test_product_path_refuses_without_device():
    from evolutionarydistributedtraining_amd import EdtError, ops
    if torch.cuda.is_available():
        pytest.skip("a GPU is visible")
    with pytest.raises(EdtError):
        ops.outer_step(torch.zeros(8), [torch.zeros(8)], None, False, 0.7, 0.0, False)
    with pytest.raises(EdtError):
        merge.slerp(0.5, torch.zeros(4), torch.ones(4))


# public names of the reference's three crossover modules (EDT_LM/train/crossover.py,
# EDT_RL/crossover.py, EDT_EVOMERGE/train/crossover.py), as written there
REFERENCE_SURFACES = {
    "lm_crossover": ["slerp", "lerp", "maybe_torch", "normalize", "load_model_from_path", "interpolate_t",
                     "LazyTensorLoader", "run_slerp_merge_from_config", "run_linear_merge_5050", "run_sgd",
                     "crossover_main", "uniform_dna_crossover"],
    "rl_crossover": ["slerp", "lerp", "maybe_torch", "normalize", "load_model_from_folder", "interpolate_t",
                     "run_slerp_merge_from_config", "run_slerp_merge", "uniform_crossover", "crossover"],
    "evomerge_crossover": ["slerp", "lerp", "maybe_torch", "normalize", "load_model_from_path", "interpolate_t",
                           "LazyTensorLoader", "run_slerp_merge_from_config", "run_linear_merge_5050",
                           "crossover_main", "uniform_dna_crossover"],
}


@pytest.mark.parametrize("mod", sorted(REFERENCE_SURFACES))
def test_every_reference_name_is_mirrored(mod):
    import importlib
    m = importlib.import_module(f"evolutionarydistributedtraining_amd.{mod}")
    for name in REFERENCE_SURFACES[mod]:
        assert hasattr(m, name), f"{mod}.{name}"
        assert name in m.__all__, f"{mod}.__all__ lacks {name}"


def test_host_helpers_match_reference_semantics(oracle):
    import numpy as np
    from evolutionarydistributedtraining_amd.merge import LazyTensorLoader, maybe_torch, normalize
    v = np.random.default_rng(0).standard_normal(1000).astype(np.float32)
    assert np.array_equal(normalize(v, 1e-8), oracle._unit(v, 1e-8))
    z = np.zeros(5, dtype=np.float32)
    assert normalize(z, 1e-8) is z                          # no division below eps
    assert isinstance(maybe_torch(v, True), torch.Tensor) and maybe_torch(v, False) is v
    lin = torch.nn.Linear(3, 2)
    loader = LazyTensorLoader(lin)
    assert torch.equal(loader.get_tensor("weight"), lin.weight.detach())
    loader.flush()
    assert loader.state_dict is None


def test_sgd_argument_errors_match_torch():
    """The outer optimiser's argument checks raise what torch.optim.SGD raises (the reference
    builds one per outer step)."""
    from evolutionarydistributedtraining_amd.diloco import check_sgd_hparams
    for lr, mu, nest in [(0.7, 0.0, True), (-1.0, 0.9, False), (0.7, -0.1, False)]:
        with pytest.raises(ValueError) as ours:
            check_sgd_hparams(lr, mu, nest)
        with pytest.raises(ValueError) as theirs:
            torch.optim.SGD([torch.zeros(1, requires_grad=True)], lr=lr, momentum=mu, nesterov=nest)
        assert str(ours.value) == str(theirs.value)
    check_sgd_hparams(1.0, 0.0, False)        # diloco_sim.py defaults are valid


def test_abi_error_convention_without_device():
    """The C ABI's error convention (include/edt_sync.h: 0 or a negative EDT_ERR_*, the reason in
    edt_last_error()) for arguments the library rejects on the host before any HIP call — the
    reference raises at the same points (a Python exception, e.g. EDT_LM/train/crossover.py:227).
    Pointers here are host addresses that are never dereferenced; n = 0 (empty tensors) returns 0
    without a launch."""
    import ctypes
    from evolutionarydistributedtraining_amd import _lib
    lib = _lib.load_library()
    P = ctypes.c_void_p
    host = (ctypes.c_uint8 * 4096)()
    base = ctypes.addressof(host)
    p = [P(base + 64 * i) for i in range(32)]          # distinct 16-byte aligned fake addresses

    def arr(ptrs):
        return (P * len(ptrs))(*ptrs)

    def err(rc, needle):
        msg = lib.edt_last_error().decode()
        assert rc == -1 and needle in msg, (rc, msg)

    F32, BF16 = 0, 1
    ks = arr(p[1:9])
    # edt_outer_step (EDT_LM/diloco.py:238-289)
    err(lib.edt_outer_step(p[0], 5, ks, F32, 8, p[9], 1, 8, 0.7, 0.9, 1, None), "dtype")
    err(lib.edt_outer_step(p[0], BF16, ks, F32, 8, p[9], 1, 8, 0.7, 0.9, 1, None), "dtype")  # bf16 theta, f32 workers
    err(lib.edt_outer_step(p[0], F32, ks, F32, 0, p[9], 1, 8, 0.7, 0.9, 1, None), "worker count")
    err(lib.edt_outer_step(p[0], F32, arr(p[:1] * 65), F32, 65, p[9], 1, 8, 0.7, 0.9, 1, None), "out of range")
    err(lib.edt_outer_step(p[0], F32, arr([p[1], None, p[3]]), F32, 3, p[9], 1, 8, 0.7, 0.9, 1, None),
        "theta_k[1] is null")
    err(lib.edt_outer_step(p[0], F32, ks, F32, 8, None, 1, 8, 0.7, 0.9, 1, None), "momentum buffer is null")
    assert lib.edt_outer_step(None, F32, ks, F32, 8, None, 0, 0, 0.7, 0.0, 0, None) == 0   # empty
    assert lib.edt_last_error() == b""
    # edt_pair_merge_to (EDT_LM/train/crossover.py:166-237)
    err(lib.edt_pair_merge_to(p[1], p[2], p[3], p[4], 3, p[5], F32, p[6], p[7], 1, 8, 0.7, 0.9, 1, None), "dtype")
    err(lib.edt_pair_merge_to(None, p[2], p[3], p[4], BF16, p[5], BF16, p[6], p[7], 1, 8, 0.7, 0.9, 1, None),
        "null buffer")
    err(lib.edt_pair_merge_to(p[1], p[2], p[3], p[4], BF16, p[5], BF16, None, p[7], 1, 8, 0.7, 0.9, 1, None),
        "carried momentum is null")
    assert lib.edt_pair_merge_to(None, None, None, None, BF16, None, BF16, None, None, 0, 0, 0.7, 0.9, 1, None) == 0
    # edt_pair_merge_population: child count, and an output that is another child's input
    one = arr(p[1:2])
    err(lib.edt_pair_merge_population(one, one, one, one, BF16, one, BF16, None, None, None, 17, 8,
                                      0.7, 0.0, 0, None), "child count")
    b1, b2, m1, m2 = arr([p[1], p[2]]), arr([p[3], p[4]]), arr([p[5], p[6]]), arr([p[7], p[8]])
    err(lib.edt_pair_merge_population(b1, b2, m1, m2, BF16, arr([p[9], p[1]]), BF16, None, None, None, 2, 8,
                                      0.7, 0.0, 0, None), "child 1 writes an input of child 0")
    err(lib.edt_pair_merge_population(b1, b2, m1, m2, BF16, arr([p[9], p[9]]), BF16, None, None, None, 2, 8,
                                      0.7, 0.0, 0, None), "write the same buffer")
    # edt_lerp (crossover.py:50-51): fp32 inputs computed in bf16 is not a reference combination
    err(lib.edt_lerp(p[1], p[2], F32, p[3], F32, BF16, 8, 0.5, None), "bf16 compute of fp32")
    err(lib.edt_lerp(p[1], None, BF16, p[3], BF16, BF16, 8, 0.5, None), "null buffer")
    # the split SLERP passes and the one-call forms (EDT_RL/crossover.py:11-43): negative chunk /
    # segment counts are rejected before any grid is sized from them
    err(lib.edt_slerp_stats(p[1], p[2], BF16, p[3], -1, p[4], None), "negative")
    err(lib.edt_slerp_coef(p[1], p[2], -2, p[3], 0.9995, 1e-8, p[4], None, None), "negative")
    err(lib.edt_slerp_blend(p[1], p[2], BF16, p[3], BF16, p[4], -1, p[5], None), "negative")
    err(lib.edt_slerp_merge(p[1], p[2], BF16, p[3], BF16, p[4], -1, p[5], 1, p[6], 0.9995, 1e-8, p[7], p[8],
                            None, None), "negative")
    err(lib.edt_slerp_merge_speculative(p[1], p[2], BF16, p[3], BF16, p[4], -1, p[5], 1, p[6], 0.9995, 1e-8,
                                        p[7], p[8], None, p[9], 8, None), "negative")
    err(lib.edt_slerp_blend_children(arr(p[1:3]), 2, BF16, (ctypes.c_int32 * 2)(0, 1), 1, arr(p[5:6]), BF16, p[6],
                                     -1, p[7], 1, None), "negative")
    assert lib.edt_slerp_stats(p[1], p[2], BF16, p[3], 0, p[4], None) == 0          # no chunks: nothing to do


def test_host_code_under_asan_and_ubsan():
    """tests/asan: the CPU oracle and the host logic of libedt_sync / libedt_comm (argument
    validation, chunk and tensor tables, overlap checks, the comm error paths) built with
    -fsanitize=address,undefined (host side only) and exercised without a GPU; any report fails."""
    import subprocess
    d = os.path.join(ROOT, "tests", "asan")
    subprocess.run(["make", "-s", "-C", d], check=True, timeout=900)
    p = subprocess.run([os.path.join(d, "_build", "host_checks")], capture_output=True, text=True, timeout=300,
                       env=dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=1",
                                UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1"))
    assert p.returncode == 0 and "host checks ok" in p.stdout, p.stderr[-3000:]


@pytest.mark.parametrize("threads,vec", [(1, 32), (3, 32), (8, 16), (64, 32)])
def test_torch_tail_bits_match_the_oracle_mask(oracle, threads, vec):
    """torchcompat.torch_cpu_tail_bits (the product's restatement of torch's vectorized_loop /
    parallel_for tails, for edt_outer_step_tail) packs exactly the oracle's tail mask."""
    import numpy as np

    from evolutionarydistributedtraining_amd.torchcompat import torch_cpu_tail_bits
    numels = [70_001, 5, 0, 31, 257 * 160, 33, 1_000_003, 1]
    mask = oracle.torch_cpu_tail_mask(numels, vec_elems=vec, num_threads=threads).numpy()
    bits = torch_cpu_tail_bits(numels, vec_elems=vec, num_threads=threads).numpy()
    got = np.unpackbits(bits, bitorder="little")[:mask.size]
    assert np.array_equal(got, mask) and not np.unpackbits(bits, bitorder="little")[mask.size:].any()


@pytest.mark.parametrize("threads,vec", [(1, 32), (8, 32), (3, 16)])
def test_torch_tail_bits_per_tensor_match_the_oracle_mask(oracle, threads, vec):
    """torch_cpu_tail_bits_per_tensor (the tensor-list step's masks, r5): tensor t's bits start at
    byte offs[t] and, indexed inside the tensor, are exactly the oracle's mask of that tensor."""
    import numpy as np

    from evolutionarydistributedtraining_amd.torchcompat import torch_cpu_tail_bits_per_tensor
    numels = [70_001, 5, 0, 31, 257 * 160, 33, 1_000_003, 1]
    mask = oracle.torch_cpu_tail_mask(numels, vec_elems=vec, num_threads=threads).numpy()
    bits, offs = torch_cpu_tail_bits_per_tensor(numels, vec_elems=vec, num_threads=threads)
    allbits = np.unpackbits(bits.numpy(), bitorder="little")
    start = 0
    for n, o in zip(numels, offs):
        got = allbits[8 * o: 8 * o + n]
        assert np.array_equal(got, mask[start:start + n])
        start += n
    assert offs == [sum(-(-m // 8) for m in numels[:t]) for t in range(len(numels))]


def test_examples_import_and_model_runs_on_cpu():
    """examples/diloco_sim.py and examples/edt_sim.py import without a GPU; the tiny LM and its
    synthetic batches run on the CPU (the simulations themselves are GPU tests, test_gpu_sim.py)."""
    import sys
    sys.path.insert(0, os.path.join(ROOT, "examples"))
    import diloco_sim
    import edt_sim  # noqa: F401
    m = diloco_sim.TinyLM()
    x = diloco_sim.batch(0, "cpu", size=2)
    assert x.shape == (2, diloco_sim.CTX) and int(x.max()) < diloco_sim.VOCAB
    assert bool((x[:, 1:] == (3 * x[:, :-1] + 1) % diloco_sim.VOCAB).all())
    loss = diloco_sim.loss_of(m, x)
    assert loss.ndim == 0 and float(loss) > 0


def test_seg_table_overlap_check_matches_brute_force():
    """edt_slerp_seg_table's apart check (the single-pass list form's: a sorted-span sweep in C)
    against a pairwise check of every output byte range with every parent byte range, on random
    16-byte-aligned tensors of fp32 parents and fp32 / bf16 outputs, empty tensors included."""
    import ctypes
    import random
    from evolutionarydistributedtraining_amd import _lib as L
    lib = L.load_library()

    def brute(spans_in, spans_out):
        return not any(n and m and a < c + m and c < a + n for a, n in spans_out for c, m in spans_in)

    rnd = random.Random(5)
    base = 1 << 40
    for _ in range(3000):
        T = rnd.randint(1, 5)
        osz = rnd.choice([4, 2])
        sizes = [rnd.choice([0, 1, 4, 5, 20, 50]) for _ in range(T)]
        ptr = lambda: base + 16 * rnd.randint(0, 40)
        p0, p1, po = [ptr() for _ in range(T)], [ptr() for _ in range(T)], [ptr() for _ in range(T)]
        arr = lambda xs: (ctypes.c_void_p * T)(*xs)
        host = (ctypes.c_uint64 * (3 * T))()
        rc = lib.edt_slerp_seg_table(arr(p0), arr(p1), arr(po), T, (ctypes.c_uint64 * T)(*sizes), L.EDT_F32,
                                     L.EDT_F32 if osz == 4 else L.EDT_BF16, 1, ctypes.cast(host, ctypes.c_void_p))
        ins = [(p, 4 * n) for p, n in zip(p0 + p1, sizes + sizes)]
        outs = [(p, osz * n) for p, n in zip(po, sizes)]
        assert (rc == 0) == brute(ins, outs), (sizes, p0, p1, po, osz)


def test_writes_are_safe_matches_brute_force():
    """merge._writes_are_safe (vectorised sweep) against the rule it states, checked pairwise: an
    output may coincide exactly with its own pair's inputs; any other overlap of an output with an
    input or another output is unsafe; inputs may overlap each other."""
    import random
    rnd = random.Random(7)
    buf = torch.empty(400, dtype=torch.uint8)

    def brute(pairs, outs):
        spans = []
        for i, ((a, b), o) in enumerate(zip(pairs, outs)):
            for kind, t in (("in", a), ("in", b), ("out", o)):
                if t.numel():
                    spans.append((t.data_ptr(), t.data_ptr() + t.numel(), kind, i))
        for x in range(len(spans)):
            for y in range(len(spans)):
                if x == y:
                    continue
                (a0, e0, k0, i0), (a1, e1, k1, i1) = spans[x], spans[y]
                if k0 != "out" or not (a0 < e1 and a1 < e0):
                    continue
                if k1 == "in" and i1 == i0 and (a0, e0) == (a1, e1):
                    continue
                return False
        return True

    def view():
        a = rnd.randint(0, 380)
        return buf[a:a + rnd.choice([0, 1, 5, 20])]

    n_safe = 0
    for _ in range(4000):
        P = rnd.randint(1, 4)
        pairs = [(view(), view()) for _ in range(P)]
        outs = [pairs[i][0] if rnd.random() < 0.3 else view() for i in range(P)]
        want = brute(pairs, outs)
        assert merge._writes_are_safe(pairs, outs) == want, (pairs, outs)
        n_safe += want
    assert 200 < n_safe < 3800


def test_overlaps_any_matches_brute_force():
    import random
    rnd = random.Random(9)
    buf = torch.empty(300, dtype=torch.uint8)
    view = lambda: buf[(a := rnd.randint(0, 280)):a + rnd.choice([0, 1, 4, 16])]
    for _ in range(3000):
        outs = [view() for _ in range(rnd.randint(0, 4))]
        ins = [view() for _ in range(rnd.randint(0, 5))]
        want = any(o.numel() and i.numel() and o.data_ptr() < i.data_ptr() + i.numel()
                   and i.data_ptr() < o.data_ptr() + o.numel() for o in outs for i in ins)
        assert merge._overlaps_any(outs, ins) == bool(want)
    shapes = [(3, 5), (7,), (2, 2, 3)]
    outs = merge.fresh_outputs([torch.empty(s) for s in shapes], torch.bfloat16, "cpu")
    assert [o.shape for o in outs] == [torch.Size(s) for s in shapes]
    assert all(o.is_contiguous() and o.data_ptr() % 16 == 0 for o in outs)


def test_module_tensors_is_state_dict():
    """merge.module_tensors: state_dict's keys, order and tensors for a parameters-only module;
    state_dict itself when a module has persistent buffers, extra state or a state-dict hook."""
    from transformers import Qwen2Config, Qwen2ForCausalLM
    cfg = Qwen2Config(vocab_size=24, hidden_size=8, intermediate_size=16, num_hidden_layers=3,
                      num_attention_heads=2, num_key_value_heads=1, tie_word_embeddings=True)
    m = Qwen2ForCausalLM(cfg)
    for mod in (m, m.model):
        got, want = merge.module_tensors(mod), mod.state_dict()
        assert list(got) == list(want)
        assert all(got[k].data_ptr() == want[k].data_ptr() for k in want)
        assert all(isinstance(v, torch.nn.Parameter) for v in got.values())

    class WithBuffer(torch.nn.Module):
        def __init__(self):
            super().__init__()
            self.lin = torch.nn.Linear(2, 2)
            self.register_buffer("count", torch.zeros(1))

    class WithExtra(torch.nn.Module):
        def __init__(self):
            super().__init__()
            self.lin = torch.nn.Linear(2, 2)

        def get_extra_state(self):
            return {"x": 1}

    for mod in (WithBuffer(), torch.nn.Sequential(WithExtra())):
        assert list(merge.module_tensors(mod)) == list(mod.state_dict())
    hooked = torch.nn.Sequential(torch.nn.Linear(2, 2))
    hooked[0]._register_state_dict_hook(lambda mod, sd, prefix, local: sd.pop(prefix + "bias"))
    assert list(merge.module_tensors(hooked)) == list(hooked.state_dict()) == ["0.weight"]


def test_padded_offsets():
    offs, total = merge._padded_offsets([3, 8, 0, 9, 1])
    assert offs.tolist() == [0, 8, 16, 16, 32] and total == 40
    offs, total = merge._padded_offsets([])
    assert offs.size == 0 and total == 8


def test_binding_from_pointers_host_checks():
    """SlerpListBinding.from_pointers (merge._rebind_merge's binding: addresses in a fresh buffer
    computed before any view exists): the C table check still refuses misaligned addresses and
    a length that disagrees with the plan, and sets `apart` only when no output overlaps a parent."""
    import numpy as np
    from evolutionarydistributedtraining_amd import ops
    from evolutionarydistributedtraining_amd._lib import EdtError
    sizes = [24, 8, 40]
    plan = ops.make_slerp_plan([0, 24, 32, 72], torch.device("cpu"), relative=True)
    base = 1 << 40
    p0 = np.array([base, base + 1024, base + 2048], dtype=np.uint64)
    p1 = p0 + np.uint64(1 << 20)
    po = p0 + np.uint64(2 << 20)
    b = ops.SlerpListBinding.from_pointers(plan, p0, p1, po, torch.bfloat16, torch.bfloat16, torch.device("cpu"),
                                           keep=None)
    assert b.apart and b.table.numel() == 9
    assert b.table.view(-1, 3)[:, 2].tolist() == po.astype(np.int64).tolist()
    b = ops.SlerpListBinding.from_pointers(plan, p0, p1, p0.copy(), torch.bfloat16, torch.bfloat16,
                                           torch.device("cpu"), keep=None)     # out == own v0: two-pass only
    assert not b.apart
    po2 = po.copy()
    po2[1] = p1[2] + np.uint64(16)                  # inside another pair's v1 (40 bf16 = 80 B)
    with pytest.raises(EdtError):
        ops.SlerpListBinding.from_pointers(plan, p0, p1, po2, torch.bfloat16, torch.bfloat16,
                                           torch.device("cpu"), keep=None)
    po3 = po.copy()
    po3[2] += np.uint64(2)                          # off a 16-byte boundary
    with pytest.raises(EdtError):
        ops.SlerpListBinding.from_pointers(plan, p0, p1, po3, torch.bfloat16, torch.bfloat16,
                                           torch.device("cpu"), keep=None)
    with pytest.raises(EdtError):
        ops.SlerpListBinding.from_pointers(plan, p0[:2], p1[:2], po[:2], torch.bfloat16, torch.bfloat16,
                                           torch.device("cpu"), keep=None)
    assert sizes == plan.seg_numel.tolist()


def test_binding_from_checked_writes_the_checked_image():
    """SlerpListBinding.from_checked (merge._Bound's repeat: addresses validated before, outputs a
    fresh buffer) writes the same table image as the C-checked binding, with the single-pass form
    allowed, and refuses a plan of another segment count."""
    import numpy as np

    from evolutionarydistributedtraining_amd import ops
    ns = np.array([70001, 9, 131072, 4099, 1, 8], dtype=np.int64)
    T = len(ns)
    o = np.zeros(T, dtype=np.uint64)
    o[1:] = np.cumsum((ns + 7) // 8 * 8)[:-1].astype(np.uint64)
    p0, p1, po = [np.uint64(b << 40) + o * np.uint64(2) for b in (1, 2, 3)]

    class Plan:
        relative, nseg, seg_numel = True, T, ns
    plan = Plan()
    fast = ops.SlerpListBinding.from_checked(plan, p0, p1, po, torch.bfloat16, torch.bfloat16, None, None)
    slow = ops.SlerpListBinding.__new__(ops.SlerpListBinding)
    slow.device = None
    slow._bind(plan, p0, p1, po, torch.bfloat16, torch.bfloat16, None)
    assert slow.apart and fast.apart and torch.equal(fast.table, slow.table)
    with pytest.raises(ops.L.EdtError):
        ops.SlerpListBinding.from_checked(plan, p0[:-1], p1[:-1], po[:-1], torch.bfloat16, torch.bfloat16, None, None)


def test_table_staging_is_per_host_thread():
    """The pinned pointer-table staging of a plan (ops._table_stage) belongs to the calling host
    thread: plans are shared (merge._plan_for) and virtual-rank threads bind on one plan at once, so
    two threads never write the same staging buffer; each thread alternates its own two."""
    import threading

    from evolutionarydistributedtraining_amd import ops

    class Plan:
        pass
    plan = Plan()
    got = {}
    alive = threading.Barrier(3)                  # all three alive at once (idents are not reused)

    def run(name):
        bufs = []
        for i in range(4):
            st = ops._table_stage(plan, 12)
            bufs.append(st.data_ptr())
            ops._table_upload(plan, st, 12, None)
            if i == 1:
                alive.wait()
        got[name] = bufs
        alive.wait()

    ths = [threading.Thread(target=run, args=(i,)) for i in range(3)]
    for t in ths:
        t.start()
    for t in ths:
        t.join()
    sets = [set(v) for v in got.values()]
    assert all(len(s) == 2 for s in sets)                       # two buffers per thread, in turn
    assert all(v[0] == v[2] and v[1] == v[3] and v[0] != v[1] for v in got.values())
    assert not (sets[0] & sets[1] or sets[0] & sets[2] or sets[1] & sets[2])
    assert len(plan.__dict__["_table_stage_state"]) == 3
    import gc
    del ths, t
    gc.collect()
    assert len(plan.__dict__["_table_stage_state"]) == 0      # released with the threads
