#!/bin/bash
# r6: whole-set placement (OuterSync.place_arenas) — its GPU tests and the bench line contract,
# then the default bench line twice (two processes, two placements).
set -o pipefail
O=gpurun_out/r6h
mkdir -p $O
timeout -k 10 400 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
    tests/test_gpu_surfaces.py tests/test_gpu_bench_contract.py > $O/pytest_place.log 2>&1 \
    || { tail -40 $O/pytest_place.log; exit 1; }
tail -1 $O/pytest_place.log
for i in 1 2; do
  timeout -k 10 600 python3 -u bench.py --detail-out $O/bench${i}_detail.json > $O/bench${i}.json 2> $O/bench${i}.err || { tail -20 $O/bench${i}.err; exit 1; }
  python3 -c "
import json; d=json.load(open('$O/bench${i}.json')); r=d['roofline']
print('bench', $i, d['value'], r['kernel_ms'], r['frac'], r['unplaced_ms'], r.get('placement'), d['configs1_125m']['roofline']['frac'], d['configs1_125m'].get('placement'), len(open('$O/bench${i}.json').read()))"
done
echo done
