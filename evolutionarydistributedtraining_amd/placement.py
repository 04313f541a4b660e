"""Placement of the outer step's read-modify-write streams in HBM.

The fused DiLoCo step (edt_outer_step) reads and rewrites two streams in place — theta and the
outer momentum — while it streams the K workers. How fast it runs depends on where the momentum
buffer sits physically relative to theta (DRAM bank / channel conflicts between the two streams'
read-write traffic), which the allocator decides: on one MI355X, the same launch over the same
workers took 10.66-10.85 ms with the momentum in most separate allocations and 11.3-11.9 ms when
it came right after theta's (scripts/alloc_draws.py, profiles/r01_alloc_draws.json), and each
placement keeps its speed for the life of the allocation (3 interleaved rounds within 0.4 %).
Inside one region the workers' placement does not matter; r6 found that the region the whole
operand set lands in does (profiles/r06_set_placement_probe.jsonl: three draws of the 1.3B set,
each with its momentum placed, at 10.63 / 10.32 / 10.98 ms; at 125M likewise).

A resident run keeps its arenas for every generation, so it pays to choose the placement once, by
measurement, when the buffers are created: `place_momentum` allocates a few candidate momentum
buffers, times `edt_probe_stream` (the step's exact access pattern with a trivial body) on each,
keeps the fastest (with the momentum's contents) and frees the rest; `place_set` does that in
several regions of HBM for the whole set (theta and the workers copied there) and keeps the
fastest region. No element is computed differently; only the addresses change.
"""
from __future__ import annotations

import torch

from . import _lib as L


def probe_ms(theta: torch.Tensor, workers: list[torch.Tensor], momentum: torch.Tensor, iters: int = 3) -> float:
    """Median HIP-event time of edt_probe_stream over (theta, workers, momentum): the outer
    step's access pattern (every worker read once, theta and momentum read and rewritten)."""
    lib = L.lib()
    L.require_device(theta, momentum, *workers)
    n = theta.numel()
    if momentum.numel() != n or momentum.dtype != theta.dtype or any(w.numel() != n for w in workers):
        raise L.EdtError("probe operands must share theta's size (and momentum theta's dtype)")
    workers = workers[:L.EDT_MAX_WORKERS]        # one launch's worth: the workers' placement does not matter
    arr = L.ptr_array(workers)
    st = L.stream_ptr(theta.device)

    def call():
        L.check(lib.edt_probe_stream(L.ptr(theta), L.dtype_code(theta), arr, L.dtype_code(workers[0]),
                                     len(workers), L.ptr(momentum), n, st), "edt_probe_stream")
    call()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(iters)]
    for a, b in ev:
        a.record()
        call()
        b.record()
    torch.cuda.synchronize(theta.device)
    ts = sorted(a.elapsed_time(b) for a, b in ev)
    return ts[len(ts) // 2]


def place_momentum(theta: torch.Tensor, workers: list[torch.Tensor], momentum: torch.Tensor,
                   candidates: int = 8, iters: int = 3, spacer_bytes: int = 11 << 27):
    """Return (buffer, report): the momentum's contents in whichever of `candidates` placements
    (the current buffer + candidates - 1 fresh allocations) runs the step's access pattern
    fastest, and {"candidates", "probe_ms", "chosen"}.

    Fresh allocations made back to back land in neighbouring physical ranges and tend to share
    one fate, so fresh candidate c is preceded by a held spacer allocation of c * spacer_bytes
    (1.375 GiB steps), which spreads the candidates over the address space. Candidates are
    limited to what fits in free device memory with a quarter of it to spare. The probe perturbs
    what it rewrites (x + 1e-30 * sum, which moves exact zeros), so theta and the momentum are
    restored from copies afterwards."""
    nbytes = momentum.numel() * momentum.element_size()
    free, _ = torch.cuda.mem_get_info(momentum.device)
    budget = int(free * 0.75) - 2 * nbytes                  # the two restore copies
    fit = 1
    while fit < candidates and budget >= fit * nbytes + (fit * (fit + 1) // 2) * spacer_bytes:
        fit += 1
    if fit < 2:
        return momentum, {"candidates": 1, "probe_ms": [], "chosen": 0}
    saved_theta, saved = theta.clone(), momentum.clone()
    bufs, spacers = [momentum], []
    for c in range(1, fit):
        spacers.append(torch.empty(c * spacer_bytes, dtype=torch.uint8, device=momentum.device))
        bufs.append(torch.zeros_like(momentum))
    times = [probe_ms(theta, workers, b, iters) for b in bufs]
    best = min(range(len(bufs)), key=times.__getitem__)
    chosen = bufs[best]
    chosen.copy_(saved)
    theta.copy_(saved_theta)
    del saved, saved_theta, bufs, spacers
    return chosen, {"candidates": fit, "probe_ms": [round(t, 4) for t in times], "chosen": best}


def place_set(theta: torch.Tensor, workers: list[torch.Tensor], momentum: torch.Tensor, draws: int = 3,
              candidates: int = 8, iters: int = 3, spacer_bytes: int = 7 << 30):
    """Return (theta, workers, momentum, report): the whole operand set of the step in whichever of
    `draws` regions of HBM runs its access pattern fastest, the momentum placed inside each region
    by place_momentum. What place_momentum cannot reach: how fast a placement can be depends on the
    region the whole set landed in (r6, profiles/r06_set_placement_probe.jsonl: three draws of the
    1.3B fp32 x 8 set placed at 10.63 / 10.32 / 10.98 ms; at 125M the same, r06_config1_joint.jsonl),
    so draw d > 0 copies theta and the workers into fresh allocations behind a held spacer of
    d * spacer_bytes and places a momentum there too; the fastest draw is kept and the others freed.
    Contents are unchanged (copies), only addresses move — the caller re-points whatever held the old
    buffers (OuterSync.place_arenas re-points its arenas; modules bound to the old arenas must be
    bound again). Draws are limited to what fits in free device memory with the momentum search's
    room to spare; with one draw this is place_momentum."""
    set_bytes = theta.numel() * theta.element_size() + sum(w.numel() * w.element_size() for w in workers)
    mom_bytes = momentum.numel() * momentum.element_size()
    mom0, rep0 = place_momentum(theta, workers, momentum, candidates, iters)
    first = min(rep0["probe_ms"]) if rep0["probe_ms"] else probe_ms(theta, workers, mom0, iters)
    best = {"draw": 0, "ms": first, "set": (theta, workers, mom0), "momentum": rep0}
    report = {"draws": [{"best_ms": round(first, 4), "momentum_candidates": rep0["candidates"]}], "chosen_draw": 0}
    spacers = []
    for d in range(1, max(1, draws)):
        torch.cuda.empty_cache()                  # the previous draw's freed buffers back to the device
        free, _ = torch.cuda.mem_get_info(theta.device)
        # the new set + its spacer, with room for place_momentum's copies and candidates after it
        if free * 0.75 < set_bytes + d * spacer_bytes + 6 * mom_bytes:
            report["draws_limited_by_memory"] = d
            break
        spacers.append(torch.empty(d * spacer_bytes, dtype=torch.uint8, device=theta.device))
        th = torch.empty_like(theta).copy_(theta)
        ws = [torch.empty_like(w).copy_(w) for w in workers]
        m = torch.empty_like(mom0).copy_(mom0)
        m, rep = place_momentum(th, ws, m, candidates, iters)
        ms = min(rep["probe_ms"]) if rep["probe_ms"] else probe_ms(th, ws, m, iters)
        report["draws"].append({"best_ms": round(ms, 4), "momentum_candidates": rep["candidates"]})
        if ms < best["ms"]:
            best = {"draw": d, "ms": ms, "set": (th, ws, m), "momentum": rep}
        del th, ws, m
    del spacers
    torch.cuda.empty_cache()
    report["chosen_draw"] = best["draw"]
    report["momentum"] = best["momentum"]
    report.update({k: best["momentum"][k] for k in ("candidates", "probe_ms", "chosen")})   # place_momentum's keys
    th, ws, m = best["set"]
    return th, ws, m, report
