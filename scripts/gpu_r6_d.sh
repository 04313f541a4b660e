#!/bin/bash
# r6: the end-to-end (PCIe / checkpoint) rates and the two bf16 regimes of the step on the final
# library; each step under its own limit, chained.
set -o pipefail
O=gpurun_out/r6d
mkdir -p $O
timeout -k 10 600 python3 -u scripts/e2e_large.py --what diloco,slerp --worker-dtype bf16 > $O/e2e_bf16.jsonl 2> $O/e2e_bf16.err \
    || { tail -20 $O/e2e_bf16.err; exit 1; }
timeout -k 10 600 python3 -u scripts/e2e_checkpoint_large.py --what diloco,slerp > $O/e2e_ckpt.jsonl 2> $O/e2e_ckpt.err \
    || { tail -20 $O/e2e_ckpt.err; exit 1; }
timeout -k 10 300 python3 -u bench.py --theta-dtype bf16 --worker-dtype bf16 --ops none --cpu-baseline-seconds 2 \
    --detail-out $O/bench_all_bf16_detail.json > $O/bench_all_bf16.json 2> $O/bench_all_bf16.err || { tail -20 $O/bench_all_bf16.err; exit 1; }
timeout -k 10 300 python3 -u bench.py --worker-dtype bf16 --ops none --cpu-baseline-seconds 2 \
    --detail-out $O/bench_bf16_workers_detail.json > $O/bench_bf16_workers.json 2> $O/bench_bf16_workers.err || { tail -20 $O/bench_bf16_workers.err; exit 1; }
cut -c1-400 $O/e2e_bf16.jsonl $O/e2e_ckpt.jsonl
cut -c1-300 $O/bench_all_bf16.json $O/bench_bf16_workers.json
echo done
