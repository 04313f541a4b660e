#!/bin/bash
# r5: the end-to-end (PCIe-inclusive) rates on the final tree: pinned host arenas -> H2D -> the
# step / the 7B SLERP child -> D2H (scripts/e2e_large.py), and the checkpoint edge through
# safetensors files (scripts/e2e_checkpoint_large.py). Each step under its own limit, chained.
set -o pipefail
O=gpurun_out/r5e2e
mkdir -p $O
timeout -k 10 600 python3 -u scripts/e2e_large.py --what diloco,slerp --worker-dtype bf16 > $O/e2e_bf16.jsonl 2> $O/e2e_bf16.err \
    || { tail -20 $O/e2e_bf16.err; exit 1; }
timeout -k 10 600 python3 -u scripts/e2e_checkpoint_large.py --what diloco,slerp > $O/e2e_ckpt.jsonl 2> $O/e2e_ckpt.err \
    || { tail -20 $O/e2e_ckpt.err; exit 1; }
cat $O/e2e_bf16.jsonl | cut -c1-600
cat $O/e2e_ckpt.jsonl | cut -c1-600
