"""Why BASELINE configs[1] (125M x 8 fp32 workers resident, the fused outer step) ran 0.697 of
8 TB/s on one r5 box against 0.758-0.767 on five others (Weak 4). Three suspects, one
process, each measured on the same operands:

  placement  the step over `--draws` independent allocations of the whole set (theta, 8 workers,
             momentum), each draw preceded by a held spacer so draws spread over the address
             space; per draw: the step's HIP-event time, the stream-ceiling probe (the same access
             pattern with a trivial body), and the time after place_momentum (8 candidates);
  history    the same after the bench's 1.3B arenas were allocated, used and freed first (what the
             bench's configs1_125m sub-object gets);
  grid tail  the one-shot grid (60,762 workgroups, the shipped build) against grid-stride builds
             (64 and 32 workgroups per CU) on the same draw (build_variants/f32_bpc64.so,
             f32_bpc32.so; python scripts/kernel_variants.py --build --variants default,f32_bpc64,f32_bpc32).

    python scripts/config1_probe.py > profiles/r06_config1_probe.jsonl      # GPU box
"""
import ctypes
import json
import os
import statistics
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from evolutionarydistributedtraining_amd import _lib as L  # noqa: E402
from evolutionarydistributedtraining_amd.layouts import gpt2_small, gpt_1p3b  # noqa: E402
from evolutionarydistributedtraining_amd.placement import place_momentum, probe_ms  # noqa: E402

VDIR = os.path.join(ROOT, "build_variants")
K = 8


def event_ms(fn, n=20, warm=2):
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(n)]
    for a, b in ev:
        a.record()
        fn()
        b.record()
    torch.cuda.synchronize()
    return statistics.median(a.elapsed_time(b) for a, b in ev)


def make_set(P, dev, seed):
    g = torch.Generator(device=dev).manual_seed(seed)
    theta = torch.randn(P, generator=g, device=dev) * 0.02
    workers = [theta + torch.randn(P, generator=g, device=dev) * 1e-3 for _ in range(K)]
    mom = torch.randn(P, generator=g, device=dev) * 1e-3
    return theta, workers, mom


def stepper(lib, theta, workers, mom):
    arr = L.ptr_array(workers)
    st = L.stream_ptr(theta.device)
    return lambda: lib.edt_outer_step(L.ptr(theta), 0, arr, 0, K, L.ptr(mom), 1, theta.numel(), 0.7, 0.9, 1, st)


def bind(name):
    lib = ctypes.CDLL(os.path.join(VDIR, f"{name}.so"))
    for nm, res, args in L.SIGNATURES:
        f = getattr(lib, nm, None)
        if f is not None:
            f.restype, f.argtypes = res, args
    return lib


def measure(tag, lib, P, dev, draws, spacer_bytes=3 << 30):
    held = []
    for d in range(draws):
        if d:
            held.append(torch.empty(d * spacer_bytes, dtype=torch.uint8, device=dev))
        theta, workers, mom = make_set(P, dev, 100 + d)
        step = stepper(lib, theta, workers, mom)
        ms = event_ms(step)
        ceil = probe_ms(theta, workers, mom, iters=5)
        mom2, rep = place_momentum(theta, workers, mom, 8)
        placed = event_ms(stepper(lib, theta, workers, mom2))
        algo = 48 * P
        print(json.dumps({"case": tag, "draw": d, "P": P, "ms": round(ms, 4), "frac": round(algo / ms / 1e6 / 8000, 4),
                          "stream_ceiling_ms": round(ceil, 4), "ms_over_ceiling": round(ms / ceil, 4),
                          "placed_ms": round(placed, 4), "placed_frac": round(algo / placed / 1e6 / 8000, 4),
                          "placement": rep, "theta_addr_gib": round(theta.data_ptr() / 2**30, 3),
                          "mom_addr_gib": round(mom.data_ptr() / 2**30, 3)}), flush=True)
        held.append((theta, workers, mom, mom2))
    del held
    torch.cuda.empty_cache()


def joint(P, dev, draws=3, nth=4, nmom=6, nwork=3, spacer_bytes=3 << 29):
    """Which operand's placement sets the time: per draw, the stream-ceiling probe over a grid of
    theta x momentum candidates, and the best pair again with re-drawn worker sets."""
    for d in range(draws):
        held = [torch.empty((d + 1) * (5 << 30), dtype=torch.uint8, device=dev)]
        theta, workers, mom = make_set(P, dev, 300 + d)
        ths, moms = [theta], [mom]
        for c in range(1, nth):
            held.append(torch.empty(c * spacer_bytes, dtype=torch.uint8, device=dev))
            ths.append(theta.clone())
        for c in range(1, nmom):
            held.append(torch.empty(c * spacer_bytes, dtype=torch.uint8, device=dev))
            moms.append(mom.clone())
        grid = [[round(probe_ms(t, workers, m, iters=5), 4) for m in moms] for t in ths]
        bi, bj = min(((i, j) for i in range(nth) for j in range(nmom)), key=lambda ij: grid[ij[0]][ij[1]])
        wsets = [round(grid[bi][bj], 4)]
        for c in range(1, nwork):
            held.append(torch.empty(c * (spacer_bytes << 2), dtype=torch.uint8, device=dev))
            w2 = [w.clone() for w in workers]
            wsets.append(round(probe_ms(ths[bi], w2, moms[bj], iters=5), 4))
            held.append(w2)
        print(json.dumps({"case": "joint", "draw": d, "P": P, "theta_x_momentum_ms": grid,
                          "first_ms": grid[0][0], "momentum_only_best_ms": min(grid[0]),
                          "theta_only_best_ms": min(r[0] for r in grid), "joint_best_ms": grid[bi][bj],
                          "best_pair_with_redrawn_workers_ms": wsets}), flush=True)
        del held, theta, workers, mom, ths, moms
        torch.cuda.empty_cache()


def main():
    dev = torch.device("cuda:0")
    P = gpt2_small().total
    lib = L.lib()
    draws = int(os.environ.get("DRAWS", "5"))
    if os.environ.get("JOINT_ONLY") == "1":
        joint(P, dev)
        return
    measure("fresh", lib, P, dev, draws)
    # the bench's history: the 1.3B population allocated, stepped and freed before the 125M set
    P13 = gpt_1p3b().total
    t13, w13, m13 = make_set(P13, dev, 7)
    stepper(lib, t13, w13, m13)()
    torch.cuda.synchronize()
    del t13, w13, m13
    torch.cuda.empty_cache()
    measure("after_1p3b", lib, P, dev, 2)
    # the grid: one-shot (shipped) vs grid-stride builds, interleaved on one draw
    names = [n for n in ("default", "f32_bpc64", "f32_bpc32") if os.path.exists(os.path.join(VDIR, f"{n}.so"))]
    if names:
        theta, workers, mom = make_set(P, dev, 55)
        mom, _ = place_momentum(theta, workers, mom, 8)
        libs = {n: bind(n) for n in names}
        times = {n: [] for n in names}
        for _ in range(5):
            for n in names:
                times[n].append(event_ms(stepper(libs[n], theta, workers, mom), 10, 1))
        print(json.dumps({"case": "grid", "P": P, "median_ms": {n: round(statistics.median(v), 4) for n, v in times.items()},
                          "frac": {n: round(48 * P / statistics.median(v) / 1e6 / 8000, 4) for n, v in times.items()}}),
              flush=True)


if __name__ == "__main__":
    main()
