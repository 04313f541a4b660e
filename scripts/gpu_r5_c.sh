#!/bin/bash
# r5 step C: the whole GPU suite + smoke, then the bench's list_form sub-object (same-memory leg).
set -o pipefail
O=gpurun_out/${R5_OUT:-r5k}
mkdir -p $O
timeout -k 10 900 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests > $O/pytest_gpu.log 2>&1 \
    || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
python3 -c "import json; from evolutionarydistributedtraining_amd import ops; print(json.dumps(ops.RefDot().describe()))" > $O/refdot_host.json
timeout -k 10 120 python3 -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
timeout -k 10 600 python3 -u bench.py --steps 10 --warmup 3 --ops list_form --cpu-baseline-seconds 0 \
    --bcast-compare 0 > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python3 -c "
import json; d=json.load(open('$O/bench.json'))
r=d['roofline']; print('step', d['ms_per_step'], r['frac'], 'unplaced', r.get('unplaced_ms'), r.get('unplaced_frac'))
for k,v in d['list_form'].items():
    if isinstance(v, dict): print('list', k, json.dumps(v)[:300])
"
timeout -k 10 300 python3 -u scripts/evomerge_probe.py --rounds 8 > $O/evomerge_lineage.json 2> $O/evomerge.err || { tail -20 $O/evomerge.err; exit 1; }
cat $O/evomerge_lineage.json
timeout -k 10 300 python3 -u scripts/evomerge_host_breakdown.py --rounds 8 > $O/evomerge_host_breakdown.json 2> $O/evomerge_bd.err || { tail -20 $O/evomerge_bd.err; exit 1; }
cat $O/evomerge_host_breakdown.json
