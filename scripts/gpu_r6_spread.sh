#!/bin/bash
# r6 spread study: the headline line and configs[1] in three fresh processes on this
# box, each with its own first allocation and whole-set placement search; no other extras, so a call
# costs about a minute. Lines go to gpurun_out/spread/<host>_<i>.json; scripts/spread_summary.py
# tabulates every box's placed and first-allocation figures.
set -o pipefail
O=gpurun_out/spread${DRAWS:+_d$DRAWS}
mkdir -p $O
H=$(hostname | tr -c 'A-Za-z0-9_\n' '_')_$(date +%s)
for i in 1 2 3; do
    timeout -k 10 300 python3 -u bench.py --ops configs1_125m --cpu-baseline-seconds 0 --ops-cpu-seconds 0 \
        --kernel-trace 0 --bcast-compare 0 --place-draws ${DRAWS:-3} --detail-out $O/${H}_${i}_detail.json > $O/${H}_${i}.json 2> $O/${H}_${i}.err \
        || { tail -20 $O/${H}_${i}.err; exit 1; }
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); r=d['roofline']; c=d['configs1_125m']['roofline']; \
print(sys.argv[1], r['kernel_ms'], r['frac'], r.get('unplaced_frac'), r.get('placement', {}).get('draws_ms'), c.get('frac'), d['configs1_125m'].get('unplaced_frac'))" $O/${H}_${i}.json
done
