"""Checkpoint edge of the outer step.

The reference gathers the population with K x `from_pretrained` and broadcasts the new global
model with K x `save_pretrained` (EDT_LM/diloco.py:231-235, 302-308): per tensor Python objects,
a CPU model per replica. Here a HF checkpoint directory (`model.safetensors`, or sharded with
`model.safetensors.index.json`) is read straight into a flat parameter arena: the safetensors
header gives every tensor's byte range, runs of consecutive tensors are read with `readinto`
into pinned host staging buffers and copied host->device asynchronously on a copy stream, two
staging buffers in flight, so disk/page-cache reads overlap the PCIe transfers. Writing is the
reverse (device->pinned->file) and produces a file `safetensors`/`transformers` load unchanged.
"""
from __future__ import annotations

import json
import os
import re
import struct
import threading

import torch

from .params import ParamLayout
from .tracing import traced

_ST_DTYPES = {"F32": torch.float32, "BF16": torch.bfloat16, "F16": torch.float16, "F64": torch.float64,
              "I64": torch.int64, "I32": torch.int32, "I16": torch.int16, "I8": torch.int8, "U8": torch.uint8,
              "BOOL": torch.bool}
_ST_NAMES = {v: k for k, v in _ST_DTYPES.items()}


def read_header(path: str):
    """(header dict, byte offset of the data section) of a .safetensors file."""
    with open(path, "rb") as f:
        (n,) = struct.unpack("<Q", f.read(8))
        header = json.loads(f.read(n))
    return header, 8 + n


def checkpoint_files(model_dir: str) -> dict[str, str]:
    """tensor name -> file for a HF save_pretrained directory (single or sharded). A single
    `model.safetensors` wins over an index, as transformers resolves it: a directory holding both
    (a sharded save overwritten by a single-file one) loads the single file."""
    path = os.path.join(model_dir, "model.safetensors")
    if os.path.exists(path):
        header, _ = read_header(path)
        return {k: path for k in header if k != "__metadata__"}
    idx = os.path.join(model_dir, "model.safetensors.index.json")
    with open(idx) as f:
        wm = json.load(f)["weight_map"]
    return {k: os.path.join(model_dir, v) for k, v in wm.items()}


_SHARD_RE = re.compile(r"^model-\d+-of-\d+\.safetensors$")


def remove_stale_shards(model_dir: str) -> None:
    """Delete a sharded save's index and shard files (`model-XXXXX-of-YYYYY.safetensors`), as
    save_pretrained cleans up weight files it is not rewriting: after a single-file save into a
    worker dir that held the trained replica as shards, no reader can pick the stale shards."""
    if not os.path.isdir(model_dir):
        return
    for f in os.listdir(model_dir):
        if f == "model.safetensors.index.json" or _SHARD_RE.match(f):
            os.remove(os.path.join(model_dir, f))


class _Staging:
    """Two pinned host buffers used round-robin, each guarded by the event of its last copy,
    and the copy stream their host->device copies run on. Pooled (pinning is slow): a reader
    takes one from the pool and returns it; the events keep a reused buffer from being
    overwritten before its last copy has drained."""

    def __init__(self, nbytes: int, device):
        pin = device.type == "cuda"
        self.nbytes, self.device = nbytes, device
        self.bufs = [torch.empty(nbytes, dtype=torch.uint8, pin_memory=pin) for _ in range(2)]
        self.events = [None, None]
        self.i = 0
        self.stream = torch.cuda.Stream(device) if device.type == "cuda" else None

    def next(self):
        i = self.i
        self.i ^= 1
        if self.events[i] is not None:
            self.events[i].synchronize()
        return i, self.bufs[i]

    def record(self, i):
        if self.stream is not None:
            ev = torch.cuda.Event()
            ev.record(self.stream)
            self.events[i] = ev


_stage_pool: list[_Staging] = []
_stage_lock = threading.Lock()


def _acquire_stage(nbytes: int, device) -> _Staging:
    with _stage_lock:
        for k, st in enumerate(_stage_pool):
            if st.nbytes == nbytes and st.device == device:
                return _stage_pool.pop(k)
    return _Staging(nbytes, device)


def _release_stage(st: _Staging) -> None:
    with _stage_lock:
        if len(_stage_pool) < 32:
            _stage_pool.append(st)


def read_into_arena(model_dir: str, layout: ParamLayout, flat: torch.Tensor,
                    names: list[str] | None = None, staging_bytes: int = 64 << 20,
                    caller_stream=None, tensors: tuple[int, int] | None = None) -> torch.Tensor:
    """Fill `flat` (layout order) from a HF checkpoint directory. A checkpoint tensor whose dtype
    differs from the arena's is converted on the device after the copy (torch copy_ rounding,
    as load_state_dict does). The copies are ordered after, and the arena is ready on, the
    caller's current stream (or `caller_stream`). tensors=(t0, t1): only layout tensors
    t0..t1-1 (read_many splits a large checkpoint over several readers this way)."""
    names = names or layout.names
    if len(names) != len(layout):
        raise ValueError("layout needs a name per tensor")
    t0, t1 = tensors if tensors is not None else (0, len(layout))
    files = checkpoint_files(model_dir)
    headers = {p: read_header(p) for p in set(files.values())}
    dev = flat.device
    stage = _acquire_stage(staging_bytes, dev)
    copy_stream = stage.stream
    caller = None
    if copy_stream is not None:        # earlier kernels on the compute stream may still read `flat`
        caller = caller_stream or torch.cuda.current_stream(dev)
        copy_stream.wait_stream(caller)
    # group consecutive arena tensors that are also consecutive, same-dtype byte ranges in one file
    runs = []
    for k in range(t0, t1):
        name = names[k]
        if name not in files:
            raise KeyError(f"{name} not in checkpoint {model_dir}")
        path = files[name]
        h, base = headers[path]
        meta = h[name]
        dt = _ST_DTYPES[meta["dtype"]]
        if list(meta["shape"]) != list(layout.shapes[k]):
            raise ValueError(f"{name}: checkpoint shape {meta['shape']} != {list(layout.shapes[k])}")
        b0, b1 = meta["data_offsets"]
        r = runs[-1] if runs else None
        if r and r["path"] == path and r["dtype"] == dt and r["fend"] == base + b0 and dt == flat.dtype:
            r["fend"] = base + b1
            r["n"] += layout.numels[k]
        else:
            runs.append({"path": path, "dtype": dt, "fbeg": base + b0, "fend": base + b1,
                         "arena": layout.offsets[k], "n": layout.numels[k]})
    handles = {}
    try:
        for r in runs:
            f = handles.setdefault(r["path"], open(r["path"], "rb", buffering=0))
            res = torch.empty(0, dtype=r["dtype"]).element_size()
            done = 0
            total = r["fend"] - r["fbeg"]
            while done < total:
                i, buf = stage.next()
                nb = min(total - done, buf.numel() // res * res)
                f.seek(r["fbeg"] + done)
                mv = memoryview(buf.numpy())[:nb]
                got = f.readinto(mv)
                if got != nb:
                    raise IOError(f"short read from {r['path']}")
                src = buf[:nb].view(r["dtype"])
                a = r["arena"] + done // res
                dst = flat[a:a + nb // res]
                if copy_stream is not None:
                    with torch.cuda.stream(copy_stream):
                        dst.copy_(src, non_blocking=True) if r["dtype"] == flat.dtype else \
                            dst.copy_(src.to(dev, non_blocking=True))
                    stage.record(i)
                else:
                    dst.copy_(src)
                done += nb
    finally:
        for f in handles.values():
            f.close()
        _release_stage(stage)
    if copy_stream is not None:
        caller.wait_stream(copy_stream)
    return flat


@traced("edt/checkpoint.read_many")
def read_many(items, layout: ParamLayout, names: list[str] | None = None, threads: int = 8,
              staging_bytes: int = 64 << 20) -> None:
    """read_into_arena for several (model_dir, flat) pairs at once — the K worker checkpoints of
    a generation (EDT_LM/diloco.py:231-235 loads them one after another): one reader thread per
    checkpoint (file reads release the GIL), each with its own pinned staging pair and copy
    stream, so page-cache/disk reads of one worker overlap the PCIe copies of another. The arenas
    are ready on the caller's current stream when this returns."""
    from concurrent.futures import ThreadPoolExecutor
    items = list(items)
    if not items:
        return
    dev = items[0][1].device
    caller = torch.cuda.current_stream(dev) if dev.type == "cuda" else None
    if threads <= 1:
        for d, flat in items:
            read_into_arena(d, layout, flat, names, staging_bytes, caller)
        return
    # fewer checkpoints than readers (e.g. the two parents of a SLERP child): each checkpoint is
    # cut into ranges of whole tensors of about equal bytes, one reader each
    parts = max(1, threads // len(items))
    tasks = []
    for d, flat in items:
        cuts = [0]
        if parts > 1:
            tot = layout.total
            acc = 0
            for k, m in enumerate(layout.numels):
                acc += m
                if acc * parts >= (len(cuts)) * tot and len(cuts) < parts and k + 1 < len(layout):
                    cuts.append(k + 1)
        cuts.append(len(layout))
        tasks += [(d, flat, (a, b)) for a, b in zip(cuts[:-1], cuts[1:]) if b > a]

    def one(task):
        d, flat, rng = task
        if dev.type == "cuda":
            torch.cuda.set_device(dev)
        read_into_arena(d, layout, flat, names, staging_bytes, caller, tensors=rng)

    with ThreadPoolExecutor(max_workers=min(threads, len(tasks))) as ex:
        list(ex.map(one, tasks))


def _header_bytes(layout: ParamLayout, names, dtype, metadata) -> bytes:
    es = torch.empty(0, dtype=dtype).element_size()
    header = {"__metadata__": metadata or {"format": "pt"}}
    off = 0
    for name, shape, n in zip(names, layout.shapes, layout.numels):
        header[name] = {"dtype": _ST_NAMES[dtype], "shape": list(shape), "data_offsets": [off, off + n * es]}
        off += n * es
    hb = json.dumps(header, separators=(",", ":")).encode()
    hb += b" " * ((8 - len(hb) % 8) % 8)          # data section 8-byte aligned
    return struct.pack("<Q", len(hb)) + hb


_pinned: dict = {}


def _host_copy(flat: torch.Tensor) -> torch.Tensor:
    if flat.device.type != "cuda":
        return flat.contiguous()
    key = (flat.numel(), flat.dtype)
    host = _pinned.get(key)
    if host is None:                              # pinning is slow: keep the last buffer
        _pinned.clear()
        host = _pinned[key] = torch.empty(flat.numel(), dtype=flat.dtype, pin_memory=True)
    host.copy_(flat)                              # one device->host transfer, synchronous
    return host


_TRASH = ".edt-old-"                  # an old file renamed away by _publish, deleted in the background
_trash_seq = iter(range(1 << 62))
_deleter = None
_deleter_lock = threading.Lock()
_pending_deletes: list = []


def _unlink_quiet(path: str) -> None:
    try:
        os.remove(path)
    except FileNotFoundError:
        pass


def _defer_delete(path: str) -> None:
    global _deleter
    with _deleter_lock:
        if _deleter is None:
            import atexit
            from concurrent.futures import ThreadPoolExecutor
            _deleter = ThreadPoolExecutor(max_workers=4, thread_name_prefix="edt-unlink")
            atexit.register(flush_deletions)
        _pending_deletes[:] = [f for f in _pending_deletes if not f.done()]
        _pending_deletes.append(_deleter.submit(_unlink_quiet, path))


def flush_deletions() -> None:
    """Wait until every old file _publish renamed away has been deleted (also run at exit)."""
    with _deleter_lock:
        futs = list(_pending_deletes)
        _pending_deletes.clear()
    for f in futs:
        f.result()


def _publish(tmp: str, path: str) -> None:
    """The complete file tmp becomes path without a rename that replaces a file: ext4 (and overlay
    file systems over it, as on the GPU boxes) flushes a file's delayed allocation synchronously
    when a rename replaces an existing file (auto_da_alloc), which made the broadcast over the
    workers' trained checkpoints disk-bound — 8 x 2.6 GB in 3.2-4.1 s replacing, 0.53-0.60 s
    unlinking the old file first (profiles/r06_broadcast_write_probe.jsonl). An existing path is
    renamed away (path + .edt-old-<pid>-<n>), tmp renamed into the free name, and the old file —
    whose unlink frees gigabytes of cached pages — deleted by a background thread, off the
    caller's path (flush_deletions waits for it; old names left by a process that died first are
    deleted by the next publish into that directory). The old file stays until the new one is
    complete; the name is absent only between the two renames (the reference's in-place save
    truncates the file before writing it)."""
    d, base = os.path.split(path)
    trash = f"{path}{_TRASH}{os.getpid()}-{next(_trash_seq)}"
    try:
        os.rename(path, trash)
    except FileNotFoundError:
        trash = None
    os.rename(tmp, path)
    if trash is not None:
        _defer_delete(trash)
        prefix = base + _TRASH
        for f in os.listdir(d or "."):          # left by a process that died before deleting
            if f.startswith(prefix) and not _pid_alive(f[len(prefix):].split("-")[0]):
                _defer_delete(os.path.join(d, f))


def _pid_alive(pid: str) -> bool:
    try:
        os.kill(int(pid), 0)
    except (ValueError, ProcessLookupError):
        return False
    except PermissionError:
        return True
    return True


def copy_file(src: str, dst: str) -> None:
    """shutil.copy(src, dst) without writing over an existing dst (unlinked first: see _publish)."""
    import shutil
    try:
        os.remove(dst)
    except FileNotFoundError:
        pass
    shutil.copy(src, dst)


def _write_file(path: str, header: bytes, host: torch.Tensor, threads: int = 1, min_bytes: int = 64 << 20) -> None:
    """header + the host bytes to path (via path.tmp, renamed when complete). threads > 1: the data
    section is written by that many threads at their own offsets (os.pwrite releases the GIL)."""
    tmp = path + ".tmp"
    data = memoryview(host.view(torch.uint8).numpy())
    if threads <= 1 or len(data) < min_bytes:
        with open(tmp, "wb") as f:
            f.write(header)
            f.write(data)
    else:
        from concurrent.futures import ThreadPoolExecutor
        fd = os.open(tmp, os.O_WRONLY | os.O_CREAT | os.O_TRUNC, 0o644)
        try:
            os.pwrite(fd, header, 0)
            step = -(-len(data) // threads)
            step = -(-step // 4096) * 4096

            def part(a):
                view = data[a:a + step]
                done = 0
                while done < len(view):
                    done += os.pwrite(fd, view[done:], len(header) + a + done)
            with ThreadPoolExecutor(max_workers=threads) as ex:
                list(ex.map(part, range(0, len(data), step)))
        finally:
            os.close(fd)
    _publish(tmp, path)


def _stream_write(path: str, header: bytes, flat: torch.Tensor, staging_bytes: int, writers: int = 1) -> None:
    """header + the device arena's bytes to path (via path.tmp, renamed when complete) through
    pooled pinned staging pairs: the D2H of a writer's next chunk runs on its staging copy stream
    (after the caller's stream, so every kernel that produced `flat` has finished) while its
    current chunk is written. writers > 1: that many threads, each with its own staging pair and
    copy stream, take every writers-th chunk and write it at its own offset (os.pwrite releases
    the GIL), so page-cache copies of several chunks proceed at once."""
    from concurrent.futures import ThreadPoolExecutor
    dev = flat.device
    data = flat.view(torch.uint8)
    n = data.numel()
    caller = torch.cuda.current_stream(dev)
    chunks = list(range(0, n, staging_bytes))
    writers = max(1, min(writers, len(chunks)))
    tmp = path + ".tmp"
    fd = os.open(tmp, os.O_WRONLY | os.O_CREAT | os.O_TRUNC, 0o644)
    hl = len(header)

    def writer(w):
        with torch.cuda.device(dev):        # restores the caller's current device afterwards
            _write_chunks(w)

    def _write_chunks(w):
        stage = _acquire_stage(staging_bytes, dev)
        try:
            stage.stream.wait_stream(caller)
            mine = chunks[w::writers]
            pending = []

            def issue(s0):
                i, buf = stage.next()        # its previous chunk was written two steps ago
                nb = min(n, s0 + staging_bytes) - s0
                with torch.cuda.stream(stage.stream):
                    buf[:nb].copy_(data[s0:s0 + nb], non_blocking=True)
                stage.record(i)
                pending.append((i, buf, s0, nb))
            k = 0
            while pending or k < len(mine):
                while k < len(mine) and len(pending) < 2:
                    issue(mine[k])
                    k += 1
                i, buf, s0, nb = pending.pop(0)
                stage.events[i].synchronize()
                mv = memoryview(buf[:nb].numpy())
                done = 0
                while done < nb:
                    done += os.pwrite(fd, mv[done:], hl + s0 + done)
        finally:
            _release_stage(stage)
    try:
        done = 0
        while done < hl:
            done += os.pwrite(fd, header[done:], done)
        if writers == 1:
            writer(0)
        else:
            with ThreadPoolExecutor(max_workers=writers) as ex:
                list(ex.map(writer, range(writers)))
    finally:
        os.close(fd)
    _publish(tmp, path)


def _shard_groups(layout: ParamLayout, es: int, shard_bytes: int) -> list[tuple[int, int]]:
    """Runs of whole tensors of at most shard_bytes each (a tensor larger than that is a shard of
    its own), as save_pretrained's max_shard_size cuts them."""
    groups, t0, acc = [], 0, 0
    for k, m in enumerate(layout.numels):
        b = m * es
        if k > t0 and acc + b > shard_bytes:
            groups.append((t0, k))
            t0, acc = k, 0
        acc += b
    groups.append((t0, len(layout)))
    return groups


def write_sharded_from_arena(model_dir: str, layout: ParamLayout, flat: torch.Tensor, shard_bytes: int,
                             names: list[str] | None = None, metadata: dict | None = None,
                             staging_bytes: int = 64 << 20) -> list[str]:
    """`flat` as HF's sharded layout in model_dir: model-0000i-of-0000N.safetensors (runs of whole
    tensors of <= shard_bytes, `_shard_groups`) + model.safetensors.index.json, the shards written
    by one thread each. The page cache takes one file at ~11-12 GB/s whatever the writer count
    (profiles/HISTORY.md §B 8) but several files at once far faster, so a 7B child lands ~3x
    sooner as four shards (profiles/r06_e2e_sharded_write.jsonl). Any single-file
    model.safetensors and stale shards of another count are removed; the index is published last,
    so a reader sees either the old files or the complete new set."""
    from concurrent.futures import ThreadPoolExecutor
    names = names or layout.names
    es = flat.element_size()
    groups = _shard_groups(layout, es, shard_bytes)
    n = len(groups)
    files = [f"model-{i + 1:05d}-of-{n:05d}.safetensors" for i in range(n)]
    os.makedirs(model_dir, exist_ok=True)
    # the writer threads order their copies after the caller's current stream (not their own default)
    caller = torch.cuda.current_stream(flat.device) if flat.device.type == "cuda" else None

    def one(i):
        t0, t1 = groups[i]
        sub = ParamLayout(layout.shapes[t0:t1], names[t0:t1])
        part = flat[layout.offsets[t0]:layout.offsets[t0] + sub.total]
        header = _header_bytes(sub, sub.names, flat.dtype, metadata)
        target = os.path.join(model_dir, files[i])
        if caller is not None:
            with torch.cuda.device(part.device), torch.cuda.stream(caller):
                _stream_write(target, header, part, staging_bytes)
        else:
            _write_file(target, header, part.contiguous())
    if n > 1:
        with ThreadPoolExecutor(max_workers=n) as ex:
            list(ex.map(one, range(n)))
    else:
        one(0)
    keep = set(files)
    for f in os.listdir(model_dir):
        if f == "model.safetensors" or (_SHARD_RE.match(f) and f not in keep):
            os.remove(os.path.join(model_dir, f))
    index = {"metadata": {"total_size": layout.total * es},
             "weight_map": {nm: files[i] for i, (t0, t1) in enumerate(groups) for nm in names[t0:t1]}}
    idx = os.path.join(model_dir, "model.safetensors.index.json")
    with open(idx + ".tmp", "w") as f:
        json.dump(index, f, indent=2)
    _publish(idx + ".tmp", idx)
    return files


def write_from_arena(path: str, layout: ParamLayout, flat: torch.Tensor, names: list[str] | None = None,
                     metadata: dict | None = None, threads: int = 1, staging_bytes: int = 64 << 20,
                     writers: int = 1) -> None:
    """Write `flat` as a .safetensors file (tensors in layout order, one contiguous data section).
    A device arena streams through a pooled pinned staging pair (`staging_bytes` each), its D2H
    overlapping the writes: no whole-arena pinned buffer (pinning 14 GB for a 7B child costs
    1.1-1.2 s per process), and from a clean page cache 1.34-1.39 s against 1.55-1.61 s for one
    write of an already pinned copy (scripts/write_probe.py --ab, profiles/HISTORY.md §B 8). A host tensor
    is written directly (threads > 1: that many writers at their own offsets)."""
    header = _header_bytes(layout, names or layout.names, flat.dtype, metadata)
    if flat.device.type == "cuda":
        if not flat.is_contiguous():
            raise ValueError("write_from_arena needs a contiguous arena")
        _stream_write(path, header, flat, staging_bytes, writers)
    else:
        _write_file(path, header, flat.contiguous(), threads)


def save_to_dirs(dirs: list[str], layout: ParamLayout, flat: torch.Tensor, names=None) -> None:
    """The broadcast edge (EDT_LM/diloco.py:302-308): the new global model to every worker dir —
    one device->host copy, then the K files written by a thread pool (as the reference's
    ThreadPoolExecutor save does)."""
    from concurrent.futures import ThreadPoolExecutor
    if not dirs:
        return
    header = _header_bytes(layout, names or layout.names, flat.dtype, None)
    host = _host_copy(flat)
    for d in dirs:
        os.makedirs(d, exist_ok=True)

    def one(d):
        _write_file(os.path.join(d, "model.safetensors"), header, host)
        remove_stale_shards(d)        # the dir may hold the trained replica as index + shards
    with ThreadPoolExecutor(max_workers=min(len(dirs), 16)) as ex:
        list(ex.map(one, dirs))
