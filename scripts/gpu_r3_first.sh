#!/bin/bash
# Round 3, first GPU call: BASELINE configs[4] tests at the named shape, then the speculative SLERP
# pass vs lerp (HIP events; rocprofv3 kernel trace; one SQ counter pass).
set -u
cd "$(dirname "$0")/.."
R=$(pwd); OUT=$R/gpurun_out/r3a
mkdir -p $OUT
echo "== config4 tests"
EDT_RECORD_DIR=$OUT timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread \
    tests/test_gpu_config4.py > $OUT/pytest_config4.log 2>&1; s=$?
tail -5 $OUT/pytest_config4.log; [ $s -le 1 ] || exit $s
echo "== probe"
timeout -k 10 300 python scripts/slerp_spec_probe.py > $OUT/probe.json 2> $OUT/probe.err; s=$?
cat $OUT/probe.json; [ $s -eq 0 ] || exit $s
echo "== kernel trace"
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv \
    -d $OUT/kt -o probe -- python3 $R/scripts/slerp_spec_probe.py --rounds 3 > $OUT/kt.log 2>&1); s=$?
tail -2 $OUT/kt.log; [ $s -eq 0 ] || exit $s
echo "== SQ pass"
(cd /tmp && export TMPDIR=/tmp && timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LEVEL_WAVES GRBM_GUI_ACTIVE \
    --output-format csv -d $OUT/sq -o probe -- python3 $R/scripts/slerp_spec_probe.py --rounds 2 > $OUT/sq.log 2>&1); s=$?
tail -2 $OUT/sq.log
echo "== done $s"
