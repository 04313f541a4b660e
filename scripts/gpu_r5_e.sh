#!/bin/bash
# r5 step E: the SLERP list / binding / surface tests, the lm_population contract test, then the
# EVOMERGE probes (pinned table staging) and the lm_population sub-object at full size.
set -o pipefail
O=gpurun_out/${R5_OUT:-r5n}
mkdir -p $O
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_bench_contract.py \
    tests/test_gpu_surfaces.py tests/test_gpu_kernels.py tests/test_gpu_refdot.py \
    -k "lm_population or evomerge or list or bind or table or refdot or consumer" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 120 python3 -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 300 python3 -u scripts/evomerge_probe.py --rounds 8 > $O/evomerge_lineage.json 2> $O/evomerge.err || { tail -20 $O/evomerge.err; exit 1; }
timeout -k 10 300 python3 -u scripts/evomerge_host_breakdown.py --rounds 8 > $O/evomerge_host_breakdown.json 2> $O/evomerge_bd.err || { tail -20 $O/evomerge_bd.err; exit 1; }
timeout -k 10 400 python3 -u bench.py --steps 5 --warmup 2 --ops lm_population --cpu-baseline-seconds 0 --bcast-compare 0 \
    > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
cat $O/evomerge_lineage.json $O/evomerge_host_breakdown.json
