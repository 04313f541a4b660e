#!/bin/bash
# r5 final tree, last pass (after the per-thread plan workspaces and the line's kernel_trace): the
# whole GPU suite, smoke(), the EVOMERGE probe (with its same-memory leg), the default bench line
# (timed by the shell clock), then the same line under rocprofv3 --kernel-trace --stats.
set -o pipefail
O=gpurun_out/${R5_OUT:-r5final3}
R=$(pwd)
mkdir -p $O
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > $O/pytest_gpu.log 2>&1 \
    || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 120 python3 -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 300 python3 -u scripts/evomerge_probe.py --rounds 8 > $O/evomerge_lineage.json 2> $O/evomerge.err || { tail -20 $O/evomerge.err; exit 1; }
t0=$(date +%s)
timeout -k 10 900 python3 -u bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
echo "bench wall seconds: $(( $(date +%s) - t0 ))" | tee $O/bench_wall.txt
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv \
    -d $R/$O/bkt -o bench -- python3 $R/bench.py --cpu-baseline-seconds 2 > $R/$O/bench_under_rocprof.json 2> $R/$O/bkt.err) \
    || { tail -20 $O/bkt.err; exit 1; }
echo done
