"""Probe the checkpoint write edge of a 7.07B bf16 child (14.1 GB): where the
time of `checkpoint.write_from_arena` goes in a one-shot process (the reference's crossover CLI
writes one child per process, EDT_EVOMERGE/train/crossover.py:86-146), and which host-buffer form
writes fastest.

  pin_alloc        torch.empty(pin_memory=True) of the whole child (first write of a process)
  d2h_pinned       device -> that pinned buffer
  pageable_d2h     torch.empty (pageable, first touch) + device -> it
  write_pinned     one write() of the pinned buffer
  write_pageable   one write() of the pageable buffer
  chunked_C        2 pinned staging buffers of C bytes: D2H of chunk i+1 on a copy stream while
                   chunk i is written (pinning the staging pair included, as a fresh process pays it)
  --ab R           R interleaved rounds from a clean page cache (os.sync() first): one write of a
                   cached pinned whole copy, chunked_C, and checkpoint._stream_write with each of
                   `--writers` writer threads

    python scripts/write_probe.py [--dir DIR] [--chunks 268435456,1073741824] [--ab 3 --writers 1,2,4]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def _t(fn):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    out = fn()
    torch.cuda.synchronize()
    return time.perf_counter() - t0, out


def _write(path, hdr, mv):
    with open(path, "wb") as f:
        f.write(hdr)
        f.write(mv)
    os.remove(path)


def _chunked(path, hdr, xb, nbytes, c):
    """2 pinned staging buffers of c bytes (pinned here, as a fresh process would): the D2H of
    chunk i+1 on a copy stream while chunk i is written."""
    bufs = [torch.empty(c, dtype=torch.uint8, pin_memory=True) for _ in range(2)]
    st = torch.cuda.Stream()
    evs = [None, None]
    n = (nbytes + c - 1) // c

    def issue(i):
        b = bufs[i % 2]
        s0, s1 = i * c, min(nbytes, (i + 1) * c)
        with torch.cuda.stream(st):
            b[:s1 - s0].copy_(xb[s0:s1], non_blocking=True)
            ev = torch.cuda.Event()
            ev.record(st)
        evs[i % 2] = ev
        return s1 - s0
    with open(path, "wb") as f:
        f.write(hdr)
        sizes = [issue(0)]
        for i in range(n):
            if i + 1 < n:        # chunk i+1 lands in the buffer of chunk i-1, already written
                sizes.append(issue(i + 1))
            evs[i % 2].synchronize()
            f.write(memoryview(bufs[i % 2][:sizes[i]].numpy()))


def _phases(a, checkpoint, lay, x, hdr, path, nbytes, res):
    P = x.numel()

    def rate(t):
        return {"s": round(t, 3), "GBps": round(nbytes / t / 1e9, 2)}

    t, pinned = _t(lambda: torch.empty(P, dtype=torch.bfloat16, pin_memory=True))
    res["pin_alloc"] = rate(t)
    t, _ = _t(lambda: pinned.copy_(x))
    res["d2h_pinned"] = rate(t)
    t, _ = _t(lambda: _write(path, hdr, memoryview(pinned.view(torch.uint8).numpy())))
    res["write_pinned"] = rate(t)
    del pinned
    print(json.dumps(res), file=sys.stderr, flush=True)
    t, pageable = _t(lambda: torch.empty(P, dtype=torch.bfloat16).copy_(x))
    res["pageable_d2h"] = rate(t)
    t, _ = _t(lambda: _write(path, hdr, memoryview(pageable.view(torch.uint8).numpy())))
    res["write_pageable"] = rate(t)
    del pageable
    print(json.dumps(res), file=sys.stderr, flush=True)
    xb = x.view(torch.uint8)
    for c in [int(v) for v in a.chunks.split(",")]:
        t, _ = _t(lambda: (_chunked(path, hdr, xb, nbytes, c), os.remove(path)))
        res[f"chunked_{c >> 20}MiB"] = rate(t)
        print(json.dumps(res), file=sys.stderr, flush=True)
    t, _ = _t(lambda: checkpoint.write_from_arena(path, lay, x))
    res["write_from_arena_first"] = rate(t)
    t, _ = _t(lambda: checkpoint.write_from_arena(path, lay, x))
    res["write_from_arena_again"] = rate(t)
    os.remove(path)


def _ab(a, checkpoint, x, hdr, path, nbytes, res):
    """Interleaved rounds from a clean page cache (os.sync() first, its time reported)."""
    xb = x.view(torch.uint8)
    forms = {"whole_cached_pin": lambda: checkpoint._write_file(path, hdr, checkpoint._host_copy(x))}
    for c in [int(v) for v in a.chunks.split(",")]:
        forms[f"chunked_{c >> 20}MiB"] = lambda c=c: _chunked(path, hdr, xb, nbytes, c)
    for w in [int(v) for v in a.writers.split(",") if v]:
        forms[f"stream_64MiB_w{w}"] = lambda w=w: checkpoint._stream_write(path, hdr, x, 64 << 20, w)
    ab = {k: [] for k in forms}
    syncs = []
    for _ in range(a.ab):
        for k, fn in forms.items():
            t0 = time.perf_counter()
            os.sync()
            syncs.append(round(time.perf_counter() - t0, 2))
            t, _ = _t(fn)
            ab[k].append(round(t, 3))
            if os.path.exists(path):
                os.remove(path)
            print(k, ab[k][-1], file=sys.stderr, flush=True)
    res["ab_seconds"] = ab
    res["ab_sync_seconds"] = syncs


def main():
    from evolutionarydistributedtraining_amd import checkpoint
    from evolutionarydistributedtraining_amd.layouts import qwen2p5_7b_body
    ap = argparse.ArgumentParser()
    ap.add_argument("--dir", default=os.path.join(os.getcwd(), "write_probe_tmp"))
    ap.add_argument("--chunks", default=str(256 << 20) + "," + str(1 << 30))
    ap.add_argument("--ab", type=int, default=0, help="interleaved A/B repetitions after os.sync()")
    ap.add_argument("--writers", default="", help="--ab: also checkpoint._stream_write with these writer counts")
    ap.add_argument("--skip-phases", action="store_true", help="only the --ab comparison")
    a = ap.parse_args()
    os.makedirs(a.dir, exist_ok=True)
    lay = qwen2p5_7b_body()
    P = lay.total
    nbytes = 2 * P
    x = torch.empty(P, dtype=torch.bfloat16, device="cuda")
    x.fill_(0.5)
    hdr = checkpoint._header_bytes(lay, lay.names, x.dtype, None)
    path = os.path.join(a.dir, "child.safetensors")
    res = {"bytes": nbytes}
    if not a.skip_phases:
        _phases(a, checkpoint, lay, x, hdr, path, nbytes, res)
    if a.ab:
        _ab(a, checkpoint, x, hdr, path, nbytes, res)
    os.rmdir(a.dir)
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
