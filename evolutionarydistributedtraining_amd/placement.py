"""Placement of the outer step's read-modify-write streams in HBM.

The fused DiLoCo step (edt_outer_step) reads and rewrites two streams in place — theta and the
outer momentum — while it streams the K workers. How fast it runs depends on where the momentum
buffer sits physically relative to theta (DRAM bank / channel conflicts between the two streams'
read-write traffic), which the allocator decides: on one MI355X, the same launch over the same
workers took 10.66-10.85 ms with the momentum in most separate allocations and 11.3-11.9 ms when
it came right after theta's (scripts/alloc_draws.py, profiles/r01_alloc_draws.json), and each
placement keeps its speed for the life of the allocation (3 interleaved rounds within 0.4 %).
The workers' placement does not matter.

A resident run keeps its arenas for every generation, so it pays to choose the momentum's
placement once, by measurement, when the buffer is created: `place_momentum` allocates a few
candidate buffers, times `edt_probe_stream` (the step's exact access pattern with a trivial body)
on each, keeps the fastest (with the momentum's contents) and frees the rest. No element is
computed differently; only the address changes.
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
