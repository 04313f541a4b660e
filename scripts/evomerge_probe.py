"""The EVOMERGE drop-in's merge at full size (EDT_EVOMERGE/train/crossover.py:104-146, BASELINE
configs[4]'s per-child merge): two Qwen2.5-7B-shaped causal LMs in bf16 on the GPU, model_1.model
merged with model_2.model INTO model_1 (the reference's base_model = model_1), timed as the surface
runs it — merge.slerp_into_module_ (the single pass into a fresh buffer + re-pointing model_1's
parameters) against writing into model_1's own tensors (the two-pass in-place form r3 used) — with
host work included (state_dict, the key plan, the checks, the pointer table), wall clock around a
device synchronize. Both must give the same bits. Lineage parents (model_2 = model_1 + small
noise: every tensor takes the lerp branch, as fine-tunes of one base do) or --far.

    python scripts/evomerge_probe.py [--rounds 5] [--far] [--layers 28] [--repoint]
"""
import argparse
import json
import os
import statistics
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--far", action="store_true")
    ap.add_argument("--layers", type=int, default=28)
    ap.add_argument("--profile", action="store_true", help="cProfile one merge (host time split) to stderr")
    ap.add_argument("--repoint", action="store_true", help="reset model_1 to fresh tensors (no repeat binding)")
    ap.add_argument("--same-memory", type=int, default=1,
                    help="also time the surface with both models' parameters re-pointed at views of the arena "
                         "leg's two arenas (the same parent bytes at the same addresses)")
    a = ap.parse_args()
    from transformers import Qwen2Config, Qwen2ForCausalLM

    from evolutionarydistributedtraining_amd import evomerge_crossover as ev
    from evolutionarydistributedtraining_amd import merge
    dev = torch.device("cuda:0")
    cfg = Qwen2Config(vocab_size=152064, hidden_size=3584, intermediate_size=18944, num_hidden_layers=a.layers,
                      num_attention_heads=28, num_key_value_heads=4, tie_word_embeddings=False)
    torch.set_default_dtype(torch.bfloat16)
    with torch.device(dev):
        m1 = Qwen2ForCausalLM(cfg)
        m2 = Qwen2ForCausalLM(cfg)
    torch.set_default_dtype(torch.float32)
    g = torch.Generator(device=dev).manual_seed(3)
    with torch.no_grad():
        for p1, p2 in zip(m1.model.parameters(), m2.model.parameters()):
            p1.copy_(torch.randn(p1.shape, generator=g, device=dev) * 0.02)
            noise = torch.randn(p1.shape, generator=g, device=dev) * 0.02
            p2.copy_(noise if a.far else p1.float() + noise * 0.005)
    n = sum(p.numel() for p in m1.model.parameters())
    mcfg = ev.slerp_config("a", "b", cfg.num_hidden_layers)
    keys = list(m1.model.state_dict().keys())
    plan = merge.merge_plan(keys, cfg.num_hidden_layers, mcfg)
    start = {k: v.clone() for k, v in m1.model.state_dict().items()}

    def reset():
        # the start values copied into model_1's tensors where they lie (a resident population's
        # next generation: the same modules, the previous child's memory), so the repeat binding
        # of merge_models_into_ applies; --repoint: fresh tensors every round (the uncached path)
        with torch.no_grad():
            for k, p in m1.model.named_parameters():
                if a.repoint:
                    p.data = start[k].clone()
                else:
                    p.copy_(start[k])
        torch.cuda.synchronize()

    def rebind_merge():                            # the surface minus save_pretrained
        merge.merge_models_into_(m1.model, m1.model, m2.model, mcfg, cfg.num_hidden_layers, device=dev)

    def in_place_merge():
        tsd = m1.model.state_dict()
        merge.slerp_state_dicts(m1.model.state_dict(), m2.model.state_dict(), plan, out_dtype=torch.bfloat16,
                                device=dev, out=tsd)

    outs, times = {}, {}
    for name, f in (("single_pass_rebind", rebind_merge), ("two_pass_in_place", in_place_merge)):
        ts = []
        for r in range(a.rounds + 1):
            reset()
            t0 = time.perf_counter()
            f()
            torch.cuda.synchronize()
            ts.append((time.perf_counter() - t0) * 1e3)
        times[name] = ts[1:]                       # the first call builds the cached plan
        outs[name] = torch.cat([p.detach().reshape(-1) for p in m1.model.parameters()]).view(torch.int16).clone()
    same = bool(torch.equal(outs["single_pass_rebind"], outs["two_pass_in_place"]))
    if a.profile:                                  # where the host time of one merge goes
        import cProfile
        import io
        import pstats
        reset()
        pr = cProfile.Profile()
        pr.enable()
        rebind_merge()
        torch.cuda.synchronize()
        pr.disable()
        buf = io.StringIO()
        pstats.Stats(pr, stream=buf).sort_stats("tottime").print_stats(18)
        print(buf.getvalue(), file=sys.stderr)
    # the same merge as one arena pass (the single-pass speculative kernel over two flat arenas of
    # the same bodies, HIP events): the device floor the surface is measured against
    from evolutionarydistributedtraining_amd import ops
    sd1, sd2 = m1.model.state_dict(), m2.model.state_dict()
    offs = [0]
    for k, _ in plan:
        offs.append(offs[-1] + sd1[k].numel())
    v0 = torch.cat([start[k].reshape(-1) for k, _ in plan])      # the surface's parents, as arenas
    v1 = torch.cat([sd2[k].reshape(-1) for k, _ in plan])
    del sd1, sd2
    aplan = ops.make_slerp_plan(offs, dev)
    tt = torch.tensor([t for _, t in plan], dtype=torch.float64, device=dev)
    extra = {}
    if a.same_memory and not a.repoint:
        # the surface and the arena pass over the same memory: model_2's parameters re-pointed once
        # at views of the arena v1; model_1 starts as views of v0 and then lives where the merge
        # writes it (two blocks in turn, reset in place between rounds as above); after the rounds
        # the arena pass reads model_1's block and v1 and writes the other block — exactly what
        # the surface's next round would touch
        pm1, pm2 = dict(m1.model.named_parameters()), dict(m2.model.named_parameters())
        with torch.no_grad():
            for i, (k, _) in enumerate(plan):
                if k in pm2:
                    pm2[k].data = v1[offs[i]:offs[i + 1]].view(pm2[k].shape)
                if k in pm1:
                    pm1[k].data = v0[offs[i]:offs[i + 1]].view(pm1[k].shape)
        ts, out_blocks = [], []
        for r in range(a.rounds + 2):
            reset()
            t0 = time.perf_counter()
            rebind_merge()
            torch.cuda.synchronize()
            ts.append((time.perf_counter() - t0) * 1e3)
            out_blocks.append(min(p.data_ptr() for p in m1.model.parameters()))
        times["same_memory_rebind"] = ts[2:]         # the first call binds, the second repeats it
        got = torch.cat([p.detach().reshape(-1) for p in m1.model.parameters()]).view(torch.int16)
        extra["same_memory_bit_identical"] = bool(torch.equal(got, outs["single_pass_rebind"]))
        del got
        bound = next(iter(merge._bound_cache.values()))
        extra["same_memory_packed"] = int(bound.total) == n and bound.buf.data_ptr() == out_blocks[-1]
        reset()                                      # model_1's block holds the start values again
        sm_v0 = bound.buf
        sm_out = torch.empty_like(v0)
        extra["same_memory_out_block"] = sm_out.data_ptr() in out_blocks[-3:-1]
        if extra["same_memory_packed"]:
            ev2 = []
            for r in range(a.rounds + 1):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                ops.slerp_arena(aplan, sm_v0, v1, sm_out, tt, speculate=True)
                e1.record()
                torch.cuda.synchronize()
                ev2.append(e0.elapsed_time(e1))
            times["same_memory_arena_events"] = ev2[1:]
        del sm_v0, sm_out, bound
    out = torch.empty_like(v0)
    ev = []
    for r in range(a.rounds + 1):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        ops.slerp_arena(aplan, v0, v1, out, tt, speculate=True)
        e1.record()
        torch.cuda.synchronize()
        ev.append(e0.elapsed_time(e1))
    times["arena_speculative_events"] = ev[1:]
    del v0, v1, out
    res = {k: {"median_ms": round(statistics.median(v), 3), "min_ms": round(min(v), 3),
               "TBps_algorithmic": round(6 * n / (statistics.median(v) / 1e3) / 1e12, 3)} for k, v in times.items()}
    print(json.dumps({"probe": "evomerge_surface", "params_body": n, "tensors": len(keys), "far": a.far,
                      "reset": "fresh tensors" if a.repoint else "copied in place (repeat binding)",
                      "bound_entries": len(merge._bound_cache),
                      "outputs_bit_identical": same, **extra, "results": res}))


if __name__ == "__main__":
    main()
