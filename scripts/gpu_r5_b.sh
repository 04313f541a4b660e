#!/bin/bash
# r5 step B: list-form tails + needed-sums population tests, then the bench's list_form and
# population_7b sub-objects.
set -o pipefail
O=gpurun_out/${R5_OUT:-r5h}
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread \
    tests/test_gpu_population_needed.py "tests/test_gpu_kernels.py::test_list_step_with_tails_equals_flat_tail_step" \
    "tests/test_gpu_surfaces.py::test_outer_step_surface_cpu_tails_bit_exact_with_reference" \
    "tests/test_gpu_kernels.py::test_slerp_population_pair_graphs" \
    "tests/test_gpu_kernels.py::test_slerp_population_pair_graphs_dtypes" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 600 python3 -u bench.py --steps 10 --warmup 3 --ops list_form,population_7b --cpu-baseline-seconds 0 \
    --bcast-compare 0 > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python3 -c "
import json; d=json.load(open('$O/bench.json'))
r=d['roofline']; print('step', d['ms_per_step'], r['frac'], 'unplaced', r.get('unplaced_ms'), r.get('unplaced_frac'))
for k,v in d['list_form'].items():
    if isinstance(v, dict): print('list', k, v.get('kernel_ms'), v.get('wall_ms'), v.get('roofline',{}).get('frac'))
p=d['population_slerp_7b']
for f in ('speculative','two_pass'): print(f, p[f]['ms_per_generation'], p[f]['roofline']['achieved'], p[f]['roofline']['frac'])
for g in p['generations']: print(g['scale'], g['distinct_parents'], g['speculative']['ms'], g['two_pass']['ms'])
print('ring', p['ring']['speculative']['ms'], p['ring']['two_pass']['ms'])
"
