#!/bin/bash
# r6 final tree (after scripts/gpu_r6_pmc.sh stamped profiles/pmc_traffic.json for this library):
# GPU suite, smoke(), the default bench line (shell clock; its sidecar), the same line under
# rocprofv3 --kernel-trace --stats, and the kernel trace grouped by grid.
set -o pipefail
O=gpurun_out/${R6_OUT:-r6final}
R=$(pwd)
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > $O/pytest_gpu.log 2>&1 \
    || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 120 python3 -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
t0=$(date +%s)
timeout -k 10 900 python3 -u bench.py --detail-out $O/bench_detail.json > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
echo "bench wall seconds: $(( $(date +%s) - t0 ))" | tee $O/bench_wall.txt
wc -c $O/bench.json
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv \
    -d $R/$O/bkt -o bench -- python3 $R/bench.py --cpu-baseline-seconds 2 --detail-out $R/$O/bench_under_rocprof_detail.json \
    > $R/$O/bench_under_rocprof.json 2> $R/$O/bkt.err) || { tail -20 $O/bkt.err; exit 1; }
python3 scripts/trace_by_grid.py $(ls $O/bkt/*kernel_trace.csv | head -1) $O/kernels_by_grid.csv > $O/kernels_by_grid.txt 2> $O/tbg.err || tail -5 $O/tbg.err
echo done
