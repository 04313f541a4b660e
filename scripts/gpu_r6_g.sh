#!/bin/bash
# r6: whole-set placement draws at 1.3B and 125M (scripts/set_placement_probe.py).
set -o pipefail
O=gpurun_out/r6g
mkdir -p $O
timeout -k 10 400 python3 -u scripts/set_placement_probe.py > $O/set_1p3b.jsonl 2> $O/set_1p3b.err || { tail -20 $O/set_1p3b.err; exit 1; }
LAYOUT=gpt2_small DRAWS=6 SPACER_GIB=3 timeout -k 10 300 python3 -u scripts/set_placement_probe.py > $O/set_125m.jsonl 2> $O/set_125m.err || { tail -20 $O/set_125m.err; exit 1; }
cut -c1-400 $O/set_1p3b.jsonl $O/set_125m.jsonl
echo done
