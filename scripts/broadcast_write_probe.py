"""The broadcast edge's file writes (EDT_LM/diloco.py:302-308: the new global model saved into every
worker's dir): K files of identical bytes. How fast can K copies land on this file system?

  write      K files written from the host buffer by K threads (checkpoint.save_to_dirs today)
  copy       one file written, then K - 1 in-kernel copies of it (os.copy_file_range: no user-space
             pass; a file system with reflinks may share the extents copy-on-write) — K independent
             files either way, the reference's semantics
  link       one file written, then K - 1 hard links (one inode: NOT the reference's semantics; for
             comparison only)
  write_replace  as write, over K existing files written and flushed just before (the outer step
             replaces the workers' trained checkpoints)
  unlink_write  as write_replace, each existing file unlinked first (the rename then replaces
             nothing)
  publish    as write_replace, the new file complete before the old one is unlinked and the new
             one renamed into place (checkpoint._publish, r6)

Files of --mib MiB (default: the 1.3B bf16 model, 2,510 MiB) in --dir (default $TMPDIR), page cache
warm (no fsync: the best case of a shared disk, as profiles/r06_e2e_checkpoint_edge.jsonl); each
form twice, files removed between. CPU only.

    python scripts/broadcast_write_probe.py [--dir D] [--k 8] [--mib 2510] > profiles/r06_broadcast_write_probe.jsonl
"""
import argparse
import json
import os
import shutil
import tempfile
import time
from concurrent.futures import ThreadPoolExecutor

import numpy as np


def fs_type(path):
    best, kind = "", "?"
    with open("/proc/mounts") as f:
        for line in f:
            parts = line.split()
            if len(parts) > 2 and os.path.abspath(path).startswith(parts[1]) and len(parts[1]) > len(best):
                best, kind = parts[1], parts[2]
    return kind


def write_one(path, data):
    with open(path + ".tmp", "wb") as f:
        f.write(data)
    os.replace(path + ".tmp", path)


def copy_one(src, dst):
    n = os.path.getsize(src)
    with open(src, "rb") as fi, open(dst + ".tmp", "wb") as fo:
        done = 0
        while done < n:
            got = os.copy_file_range(fi.fileno(), fo.fileno(), n - done)
            if got == 0:
                raise OSError("copy_file_range made no progress")
            done += got
    os.replace(dst + ".tmp", dst)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--dir", default=os.environ.get("TMPDIR", "/tmp"))
    ap.add_argument("--k", type=int, default=8)
    ap.add_argument("--mib", type=int, default=2510)
    a = ap.parse_args()
    root = tempfile.mkdtemp(prefix="edt_bcast_", dir=a.dir)
    try:
        data = memoryview(np.random.default_rng(1).integers(0, 255, a.mib << 20, dtype=np.uint8))
        paths = [os.path.join(root, f"w{k}.safetensors") for k in range(a.k)]
        nbytes = a.k * len(data)
        print(json.dumps({"dir": root, "fs": fs_type(root), "k": a.k, "file_bytes": len(data)}), flush=True)

        def clean():
            for p in paths:
                if os.path.exists(p):
                    os.remove(p)
            os.sync()

        forms = {
            "write": lambda: list(ThreadPoolExecutor(a.k).map(lambda p: write_one(p, data), paths)),
            "copy": lambda: (write_one(paths[0], data),
                             list(ThreadPoolExecutor(a.k).map(lambda p: copy_one(paths[0], p), paths[1:]))),
            "link": lambda: (write_one(paths[0], data), [os.link(paths[0], p) for p in paths[1:]]),
        }
        def prefill():                    # the workers' trained files already there, flushed
            clean()
            list(ThreadPoolExecutor(a.k).map(lambda p: write_one(p, data), paths))
            os.sync()

        forms["write_replace"] = lambda: list(ThreadPoolExecutor(a.k).map(lambda p: write_one(p, data), paths))

        def unlink_then_write(p):
            os.remove(p)
            write_one(p, data)
        forms["unlink_write"] = lambda: list(ThreadPoolExecutor(a.k).map(unlink_then_write, paths))

        def publish(p):                   # checkpoint._publish's order: tmp complete, unlink, rename
            with open(p + ".tmp", "wb") as f:
                f.write(data)
            os.remove(p)
            os.rename(p + ".tmp", p)
        forms["publish"] = lambda: list(ThreadPoolExecutor(a.k).map(publish, paths))
        for rep in range(2):
            for name, fn in forms.items():
                prefill() if name in ("write_replace", "unlink_write", "publish") else clean()
                t0 = time.perf_counter()
                try:
                    fn()
                    s = time.perf_counter() - t0
                    rec = {"form": name, "rep": rep, "s": round(s, 3), "GBps": round(nbytes / s / 1e9, 2)}
                except OSError as e:
                    rec = {"form": name, "rep": rep, "error": f"{type(e).__name__}: {e}"}
                print(json.dumps(rec), flush=True)
    finally:
        shutil.rmtree(root, ignore_errors=True)


if __name__ == "__main__":
    main()
