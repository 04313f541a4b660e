"""Where the EVOMERGE surface's host time goes before its launch (7B Qwen2 bodies on the device):
merge.merge_models_into_'s steps called one by one, each timed with perf_counter (no device
synchronisation between them, as in the surface), the kernels' time by HIP events, several
rounds. Companion to scripts/evomerge_probe.py (which times the surface as a whole).

    python scripts/evomerge_host_breakdown.py [--rounds 5] [--layers 28]
"""
import argparse
import json
import os
import statistics
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--layers", type=int, default=28)
    a = ap.parse_args()
    from transformers import Qwen2Config, Qwen2ForCausalLM

    from evolutionarydistributedtraining_amd import evomerge_crossover as ev
    from evolutionarydistributedtraining_amd import merge, ops
    dev = torch.device("cuda:0")
    cfg = Qwen2Config(vocab_size=152064, hidden_size=3584, intermediate_size=18944, num_hidden_layers=a.layers,
                      num_attention_heads=28, num_key_value_heads=4, tie_word_embeddings=False)
    torch.set_default_dtype(torch.bfloat16)
    with torch.device(dev):
        m1 = Qwen2ForCausalLM(cfg).model
        m2 = Qwen2ForCausalLM(cfg).model
    torch.set_default_dtype(torch.float32)
    with torch.no_grad():
        for p1, p2 in zip(m1.parameters(), m2.parameters()):
            p2.copy_(p1.float() + 1e-4)
    mcfg = ev.slerp_config("a", "b", cfg.num_hidden_layers)
    steps = {}

    def t(name, t0):
        now = time.perf_counter()
        steps.setdefault(name, []).append((now - t0) * 1e3)
        return now

    for r in range(a.rounds + 1):
        torch.cuda.synchronize()
        t0 = t_start = time.perf_counter()
        sd1 = merge.module_tensors(m1)
        t0 = t("walk model_1", t0)
        sd2 = merge.module_tensors(m2)
        t0 = t("walk model_2", t0)
        plan = merge.merge_plan(list(sd1.keys()), cfg.num_hidden_layers, mcfg)
        keys = [k for k, _ in plan]
        outs = [sd1[k] for k in keys]
        t0 = t("key plan + lists", t0)
        pairs = [(sd1[k], sd2[k]) for k in keys]
        p0, p1, ns, in_dt = merge._pair_pointers(pairs, dev)
        t0 = t("pair checks + addresses", t0)
        offs, total = merge._padded_offsets(ns)
        buf = torch.empty(total, dtype=torch.bfloat16, device=dev)
        po = np.uint64(buf.data_ptr()) + offs.astype(np.uint64) * np.uint64(2)
        offsets = [0] + np.cumsum(ns).tolist()
        splan = merge._plan_for(offsets, dev, relative=True)
        t0 = t("fresh buffer + plan lookup", t0)
        tt = torch.tensor([x for _, x in plan], dtype=torch.float64).to(dev)
        t0 = t("t upload", t0)
        b = ops.SlerpListBinding.from_pointers(splan, p0, p1, po, in_dt, torch.bfloat16, dev, keep=(buf, pairs))
        t0 = t("binding (C checks + table upload)", t0)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        b.merge(tt)
        e1.record()
        t0 = t("merge launches", t0)
        with torch.no_grad():
            for k, o, off in zip(keys, outs, offs.tolist()):
                m1.get_parameter(k).data = buf.as_strided(o.shape, merge._contig_strides(o.shape), off)
        t0 = t("views + re-pointing (after the launch)", t0)
        torch.cuda.synchronize()
        t("wall", t_start)
        steps.setdefault("device (events)", []).append(e0.elapsed_time(e1))
    res = {k: round(statistics.median(v[1:]), 4) for k, v in steps.items()}
    pre = sum(v for k, v in res.items() if k not in ("wall", "device (events)", "views + re-pointing (after the launch)"))

    # the repeat of the merge through merge_models_into_'s cached binding (merge._Bound), its steps
    # one by one as merge._bound_merge runs them
    merge.clear_merge_cache()
    merge.merge_models_into_(m1, m1, m2, mcfg, cfg.num_hidden_layers, device=dev)
    torch.cuda.synchronize()
    steps = {}
    for r in range(a.rounds + 1):
        torch.cuda.synchronize()
        t0 = t_start = time.perf_counter()
        key = merge._bound_key(m1, m1, m2, mcfg, cfg.num_hidden_layers, dev)
        b = merge._bound_cache[key]
        assert b.r1() is m1 and b.r2() is m2
        t0 = t("cache key + lookup", t0)
        buf = torch.empty(b.total, dtype=b.out_dt, device=b.dev)
        po = np.uint64(buf.data_ptr()) + b.offs_bytes
        t0 = t("fresh buffer", t0)
        bd = ops.SlerpListBinding.from_checked(b.splan, b.p0, b.p1, po, b.in_dt, b.out_dt, b.dev, keep=(buf, b.buf, b.hold2))
        t0 = t("binding (C checks + table upload)", t0)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        bd.merge(b.tt)
        e1.record()
        t0 = t("merge launches", t0)
        sd1, sd2 = merge.module_tensors(m1), merge.module_tensors(m2)
        pairs = [(sd1[k], sd2[k]) for k in b.keys]
        meta = merge._pair_pointers(pairs, b.dev)
        ok = np.array_equal(meta[0], b.p0) and np.array_equal(meta[1], b.p1)
        t0 = t("module check (after the launch)", t0)
        cur = torch.cuda.current_stream(b.dev)
        with torch.no_grad():
            for k, shp, st, off in zip(b.keys, b.shapes, b.strides, b.offs_list):
                p = sd1[k]
                p.data.record_stream(cur)
                p.data = buf.as_strided(shp, st, off)
        b.p0, b.buf = po, buf
        t0 = t("re-pointing (after the launch)", t0)
        torch.cuda.synchronize()
        t("wall", t_start)
        steps.setdefault("device (events)", []).append(e0.elapsed_time(e1))
        assert ok
    bres = {k: round(statistics.median(v[1:]), 4) for k, v in steps.items()}
    bpre = sum(v for k, v in bres.items() if k in ("cache key + lookup", "fresh buffer", "binding (C checks + table upload)",
                                                   "merge launches"))
    print(json.dumps({"probe": "evomerge_host_breakdown", "median_ms": res, "host_before_launch_ms": round(pre, 4),
                      "repeat_binding": {"median_ms": bres, "host_before_launch_ms": round(bpre, 4)}}))


if __name__ == "__main__":
    main()
