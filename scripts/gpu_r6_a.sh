#!/bin/bash
# r6 first call: the GPU suite on the source-determined build, the store-kind probe (lerp and the
# pair merge at 1.3B and 7B, ordinary vs non-temporal), the configs[1] probe (placement draws,
# history, grid), and the default bench line in its capped form with its sidecar.
set -o pipefail
O=gpurun_out/r6a
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > $O/pytest_gpu.log 2>&1 \
    || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 300 python3 -u scripts/lerp7b_nt_probe.py > $O/nt_probe.jsonl 2> $O/nt_probe.err || { tail -20 $O/nt_probe.err; exit 1; }
cat $O/nt_probe.jsonl
timeout -k 10 300 python3 -u scripts/config1_probe.py > $O/config1_probe.jsonl 2> $O/config1_probe.err || { tail -20 $O/config1_probe.err; exit 1; }
cat $O/config1_probe.jsonl | cut -c1-400
t0=$(date +%s)
timeout -k 10 900 python3 -u bench.py --detail-out $O/bench_detail.json > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
echo "bench wall seconds: $(( $(date +%s) - t0 ))" | tee $O/bench_wall.txt
wc -c $O/bench.json
echo done
