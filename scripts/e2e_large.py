"""End-to-end (PCIe-inclusive) rates at the north star's sizes: the population arrives from host
memory and the result goes back, as in real runs where launch_to_machines.py's hosts hand over
checkpoints (EDT_LM/diloco.py:231-235 gather, :302-308 broadcast; EDT_EVOMERGE/train/
crossover.py:86-101 LazyTensorLoader round trip). Not the bench `value` (device-resident).

  diloco  1.3B x K workers (pinned host) -> H2D -> fused outer step -> D2H of the new theta.
          serial: every copy, then the kernel, then the copy back; pipelined: buckets, H2D of
          bucket b+1 (copy stream) || kernel on bucket b (compute stream) || D2H of bucket b-1
          (third stream).
  slerp   one SLERP child of two 7.07B bf16 bodies (qwen2p5_7b_body, t = 0.5): serial (both
          parents H2D, edt_slerp_merge, child D2H) and pipelined by groups of whole tensors
          (~1 GiB: a tensor's dot needs all of it), group g+1 H2D || merge of g || D2H of g-1.

    python scripts/e2e_large.py --what diloco,slerp [--k 8 --worker-dtype bf16]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
DT = {"f32": torch.float32, "bf16": torch.bfloat16}


def _pinned_randn(n, dtype, base=None, scale=0.02, seed=0):
    out = torch.empty(n, dtype=dtype, pin_memory=True)
    g = torch.Generator().manual_seed(seed)
    step = 1 << 26
    for s in range(0, n, step):
        e = min(n, s + step)
        x = torch.randn(e - s, generator=g) * scale
        if base is not None:
            x += base[s:e].float()
        out[s:e] = x.to(dtype)
    return out


def _time(fn, reps):
    fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        ts.append(time.perf_counter() - t0)
    return min(ts)


def diloco(a, dev):
    from evolutionarydistributedtraining_amd import ops
    from evolutionarydistributedtraining_amd.layouts import LAYOUTS
    P = LAYOUTS[a.layout]().total
    wdt = DT[a.worker_dtype]
    theta_h = _pinned_randn(P, torch.float32, seed=1)
    workers_h = [_pinned_randn(P, wdt, base=theta_h, scale=1e-3, seed=10 + k) for k in range(a.k)]
    out_h = torch.empty(P, dtype=torch.float32, pin_memory=True)
    theta_d = torch.empty(P, device=dev)
    mom_d = torch.zeros(P, device=dev)
    workers_d = [torch.empty(P, dtype=wdt, device=dev) for _ in range(a.k)]
    wb = torch.finfo(wdt).bits // 8
    metric = a.k * P * wb
    pcie = metric + 8 * P            # workers + theta in, theta out
    comp = torch.cuda.current_stream(dev)
    h2d, d2h = torch.cuda.Stream(dev), torch.cuda.Stream(dev)

    def serial():
        theta_d.copy_(theta_h, non_blocking=True)
        for wd, wh in zip(workers_d, workers_h):
            wd.copy_(wh, non_blocking=True)
        ops.outer_step(theta_d, workers_d, mom_d, True, 0.7, 0.9, True)
        out_h.copy_(theta_d, non_blocking=True)

    def pipelined():
        B = a.bucket_elems
        evs = []
        for s in range(0, P, B):
            e = min(P, s + B)
            with torch.cuda.stream(h2d):
                theta_d[s:e].copy_(theta_h[s:e], non_blocking=True)
                for wd, wh in zip(workers_d, workers_h):
                    wd[s:e].copy_(wh[s:e], non_blocking=True)
                ev = torch.cuda.Event()
                ev.record(h2d)
            evs.append((s, e, ev))
        for s, e, ev in evs:
            comp.wait_event(ev)
            ops.outer_step(theta_d[s:e], [w[s:e] for w in workers_d], mom_d[s:e], True, 0.7, 0.9, True)
            done = torch.cuda.Event()
            done.record(comp)
            d2h.wait_event(done)
            with torch.cuda.stream(d2h):
                out_h[s:e].copy_(theta_d[s:e], non_blocking=True)
        comp.wait_stream(d2h)

    res = {"layout": a.layout, "P": P, "K": a.k, "worker_dtype": a.worker_dtype, "bucket_elems": a.bucket_elems,
           "pcie_bytes": pcie, "metric_bytes": metric}
    for name, fn in (("serial", serial), ("pipelined", pipelined)):
        t = _time(fn, a.reps)
        res[name] = {"ms": round(t * 1e3, 1), "metric_GBps": round(metric / t / 1e9, 2),
                     "pcie_GBps": round(pcie / t / 1e9, 2)}
    tk = _time(lambda: ops.outer_step(theta_d, workers_d, mom_d, True, 0.7, 0.9, True), a.reps)
    res["device_resident"] = {"ms": round(tk * 1e3, 2), "metric_GBps": round(metric / tk / 1e9, 1)}
    # the copies alone (host -> device of everything, device -> host of theta)
    th = _time(lambda: [theta_d.copy_(theta_h, non_blocking=True)] +
               [wd.copy_(wh, non_blocking=True) for wd, wh in zip(workers_d, workers_h)], a.reps)
    res["h2d_only"] = {"ms": round(th * 1e3, 1), "GBps": round((metric + 4 * P) / th / 1e9, 2)}
    return res


def slerp(a, dev):
    from evolutionarydistributedtraining_amd import ops
    from evolutionarydistributedtraining_amd.layouts import qwen2p5_7b_body
    lay = qwen2p5_7b_body()
    P, bf = lay.total, torch.bfloat16
    v0_h = _pinned_randn(P, bf, seed=3)
    v1_h = _pinned_randn(P, bf, base=v0_h, scale=1e-3, seed=4)       # far parents: the SLERP branch
    out_h = torch.empty(P, dtype=bf, pin_memory=True)
    v0, v1, out = (torch.empty(P, dtype=bf, device=dev) for _ in range(3))
    t_all = torch.full((len(lay),), 0.5, dtype=torch.float64, device=dev)
    plan = ops.make_slerp_plan(lay.offsets, dev)
    # groups of whole tensors of ~group_bytes, each with its own plan over offsets relative to it
    offs = lay.offsets
    groups, g0 = [], 0
    for i in range(1, len(offs)):
        if (offs[i] - offs[g0]) * 2 >= a.group_bytes or i == len(offs) - 1:
            groups.append((g0, i))
            g0 = i
    gplans = [ops.make_slerp_plan([o - offs[s] for o in offs[s:e + 1]], dev) for s, e in groups]
    comp = torch.cuda.current_stream(dev)
    h2d, d2h = torch.cuda.Stream(dev), torch.cuda.Stream(dev)

    def serial():
        v0.copy_(v0_h, non_blocking=True)
        v1.copy_(v1_h, non_blocking=True)
        ops.slerp_arena(plan, v0, v1, out, t_all)
        out_h.copy_(out, non_blocking=True)

    def pipelined():
        evs = []
        for s, e in groups:
            a0, a1 = offs[s], offs[e]
            with torch.cuda.stream(h2d):
                v0[a0:a1].copy_(v0_h[a0:a1], non_blocking=True)
                v1[a0:a1].copy_(v1_h[a0:a1], non_blocking=True)
                ev = torch.cuda.Event()
                ev.record(h2d)
            evs.append(ev)
        for (s, e), gp, ev in zip(groups, gplans, evs):
            a0, a1 = offs[s], offs[e]
            comp.wait_event(ev)
            ops.slerp_arena(gp, v0[a0:a1], v1[a0:a1], out[a0:a1], t_all[s:e])
            done = torch.cuda.Event()
            done.record(comp)
            d2h.wait_event(done)
            with torch.cuda.stream(d2h):
                out_h[a0:a1].copy_(out[a0:a1], non_blocking=True)
        comp.wait_stream(d2h)

    res = {"layout": "qwen2p5_7b_body", "P": P, "groups": len(groups), "pcie_bytes": 6 * P,
           "algo_bytes": 6 * P}
    for name, fn in (("serial", serial), ("pipelined", pipelined)):
        t = _time(fn, a.reps)
        res[name] = {"ms": round(t * 1e3, 1), "pcie_GBps": round(6 * P / t / 1e9, 2)}
    tk = _time(lambda: ops.slerp_arena(plan, v0, v1, out, t_all), a.reps)
    res["device_resident"] = {"ms": round(tk * 1e3, 2), "algo_GBps": round(6 * P / tk / 1e9, 1),
                              "form": "speculative" if ops._speculation_pays(plan, 2, 2) else "two_pass"}
    # both pipelined forms must give the device-resident child
    pipelined()
    torch.cuda.synchronize()
    ref = out.clone()
    ops.slerp_arena(plan, v0, v1, out, t_all, speculate=False)
    torch.cuda.synchronize()
    res["pipelined_equals_whole_arena"] = bool(torch.equal(ref.view(torch.int16), out.view(torch.int16)))
    return res


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--what", default="diloco,slerp")
    ap.add_argument("--layout", default="gpt_1p3b")
    ap.add_argument("--k", type=int, default=8)
    ap.add_argument("--worker-dtype", default="bf16", choices=DT)
    ap.add_argument("--bucket-elems", type=int, default=1 << 26)
    ap.add_argument("--group-bytes", type=int, default=1 << 30)
    ap.add_argument("--reps", type=int, default=3)
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    out = {}
    if "diloco" in a.what:
        out["diloco"] = diloco(a, dev)
        torch.cuda.empty_cache()
        print(json.dumps(out["diloco"]), flush=True)
    if "slerp" in a.what:
        out["slerp"] = slerp(a, dev)
        print(json.dumps(out["slerp"]), flush=True)


if __name__ == "__main__":
    main()
