#!/bin/bash
# bench.py after the ExtrasDeadline restructure: the N=1 line, the multi-GPU code path at world 1
# (--sharded: every extra, CPU baseline before them), and the same with a 3-s deadline that fires
# inside the extras (the line must still print, exit status 0). Each GPU step under its own limit.
set -u
cd "$(dirname "$0")/.."
OUT=gpurun_out; mkdir -p $OUT
timeout -k 10 300 python bench.py > $OUT/dl_n1.log 2>&1 || exit $?
grep '^{' $OUT/dl_n1.log > $OUT/dl_n1.json
timeout -k 10 400 python bench.py --gpus 1 --sharded > $OUT/dl_sharded.log 2>&1 || exit $?
grep '^{' $OUT/dl_sharded.log > $OUT/dl_sharded.json
timeout -k 10 200 python bench.py --gpus 1 --sharded --extras-deadline 3 > $OUT/dl_fire.log 2>&1; s=$?
echo "deadline run exit status $s"
grep '^{' $OUT/dl_fire.log > $OUT/dl_fire.json || exit 1
python - <<'EOF'
import json
for f in ("dl_n1", "dl_sharded", "dl_fire"):
    d = json.load(open(f"gpurun_out/{f}.json"))
    print(f, d["value"], d["ms_per_step"], sorted(d), d.get("extras_deadline"))
EOF
exit $s
