"""Where the reference's torch CPU kernels round differently: the scalar tails.

torch's CPU binary kernels (aten/native/cpu/Loops.h `vectorized_loop`) process each contiguous run
Vec::size() elements at a time and the last `run % Vec::size()` elements one by one; the runs are
the chunks at::parallel_for hands to its threads (grain 32768: a tensor of n elements is cut into
min(threads, ceil(n / grain)) chunks of ceil(n / chunks)). For `add(x, y, alpha)` in bf16 the
vectorised path is one fp32 FMA rounded once and the scalar path rounds alpha * y first — the two
alpha-adds of the reference's SGD step (EDT_LM/diloco.py:252-289, EDT_LM/train/crossover.py:
228-230) differ by up to one bf16 ulp on those elements. `torch_cpu_tail_bits` gives the kernels
(edt_outer_step_tail / edt_pair_merge_tail) the tail elements of a given host, so a bf16 step can
be bit-exact with the reference as run there (Vec::size() = 32 bf16 on AVX-512, 16 on AVX2;
threads = torch.get_num_threads() on the reference's master)."""
from __future__ import annotations

import numpy as np
import torch

TORCH_GRAIN = 32768


def torch_cpu_tail_ranges(numels, vec_elems: int = 32, num_threads: int = 1, grain: int = TORCH_GRAIN):
    """[start, end) of every scalar-tail run of a flat concatenation of tensors of sizes `numels`."""
    out, off = [], 0
    for n in numels:
        n = int(n)
        if n:
            tasks = max(1, min(num_threads, -(-n // grain)))
            chunk = -(-n // tasks)
            for b in range(0, n, chunk):
                e = min(n, b + chunk)
                t0 = b + (e - b) // vec_elems * vec_elems
                if t0 < e:
                    out.append((off + t0, off + e))
        off += n
    return out


def torch_cpu_tail_bits(numels, vec_elems: int = 32, num_threads: int = 1, grain: int = TORCH_GRAIN,
                        device=None) -> torch.Tensor:
    """The tail elements as a bitmask (uint8, bit i & 7 of byte i >> 3), ceil(total / 8) bytes."""
    total = int(sum(int(n) for n in numels))
    mask = np.zeros(max(1, -(-total // 8)) * 8, dtype=np.uint8)
    for a, b in torch_cpu_tail_ranges(numels, vec_elems, num_threads, grain):
        mask[a:b] = 1
    bits = torch.from_numpy(np.packbits(mask, bitorder="little"))
    return bits.to(device) if device is not None else bits


def torch_cpu_tail_bits_per_tensor(numels, vec_elems: int = 32, num_threads: int = 1, grain: int = TORCH_GRAIN,
                                   device=None):
    """The same tail elements for T separate tensors (the tensor-list step, edt_outer_step_list_tail):
    each tensor's bits start at a byte boundary, indexed by the element's index inside its tensor.
    Returns (bits uint8 [sum ceil(n / 8)], byte offset of each tensor's bits)."""
    parts, offs, off = [], [], 0
    for n in numels:
        n = int(n)
        nb = -(-n // 8)
        offs.append(off)
        if nb:
            mask = np.zeros(nb * 8, dtype=np.uint8)
            for a, b in torch_cpu_tail_ranges([n], vec_elems, num_threads, grain):
                mask[a:b] = 1
            parts.append(np.packbits(mask, bitorder="little"))
        off += nb
    bits = torch.from_numpy(np.concatenate(parts) if parts else np.zeros(1, dtype=np.uint8))
    return (bits.to(device) if device is not None else bits), offs
