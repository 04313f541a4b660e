#!/bin/bash
# r5 step A: needed-sums population passes — GPU parity, then the roulette probe in the legacy
# (r4 ring / triangle / co-located) and the new layout, same box.
set -o pipefail
O=gpurun_out/${R5_OUT:-r5a}
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread \
    tests/test_gpu_population_needed.py "tests/test_gpu_kernels.py::test_slerp_population_pair_graphs" \
    "tests/test_gpu_kernels.py::test_slerp_population_pair_graphs_dtypes" \
    "tests/test_gpu_kernels.py::test_slerp_population_matches_per_child" > $O/pytest_needed.log 2>&1 || { tail -30 $O/pytest_needed.log; exit 1; }
tail -3 $O/pytest_needed.log
timeout -k 10 400 python3 -u scripts/pop_roulette_probe.py --graphs 6 --rounds 3 --ring --independent \
    --out $O/pop_roulette_repeat.json > $O/pop_roulette_repeat.log 2>&1 || { tail -20 $O/pop_roulette_repeat.log; exit 1; }
timeout -k 10 400 python3 -u scripts/pop_roulette_probe.py --graphs 6 --rounds 3 --ring --independent \
    --out $O/pop_roulette_needed.json > $O/pop_roulette_needed.log 2>&1 || { tail -20 $O/pop_roulette_needed.log; exit 1; }
tail -n 2 $O/pop_roulette_repeat.log; tail -n 2 $O/pop_roulette_needed.log
