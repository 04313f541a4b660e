#!/bin/bash
# r5: the bench line's in-process kernel trace — the contract tests (N = 1 line and the multi-GPU code
# path at world 1), then a short line under rocprofv3 --kernel-trace --stats (the trace must step aside).
set -o pipefail
O=gpurun_out/r5trace
mkdir -p $O
R=$(pwd)
timeout -k 10 400 python3 -u -m pytest -x -v --timeout 150 --timeout-method thread -m gpu tests/test_gpu_bench_contract.py \
    > $O/pytest_contract.log 2>&1 || { tail -40 $O/pytest_contract.log; exit 1; }
tail -1 $O/pytest_contract.log
timeout -k 10 300 python3 -u bench.py --steps 10 --warmup 3 --ops none --cpu-baseline-seconds 1 > $O/bench_short.json 2> $O/bench_short.err \
    || { tail -20 $O/bench_short.err; exit 1; }
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$O/kt -o bench -- python3 $R/bench.py --steps 10 --warmup 3 --ops none \
    --cpu-baseline-seconds 0 --place-candidates 1 > $R/$O/bench_under_rocprof.json 2> $R/$O/bench_under_rocprof.err \
    || { tail -20 $R/$O/bench_under_rocprof.err; exit 1; }
echo done
