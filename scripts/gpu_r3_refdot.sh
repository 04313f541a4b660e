#!/bin/bash
# Round 3: reference-dot mode + the SLERP tests, then the standalone speculative-pass probe.
set -u
cd "$(dirname "$0")/.."
R=$(pwd); OUT=$R/gpurun_out/${TAG:-r3e}
mkdir -p $OUT
EDT_RECORD_DIR=$OUT timeout -k 10 900 python -u -m pytest -x -q -m gpu --timeout 300 --timeout-method thread \
    ${TESTS:-tests/test_gpu_refdot.py tests/test_slerp_threshold.py tests/test_gpu_slerp_split.py tests/test_gpu_config4.py tests/test_gpu_configs.py} \
    > $OUT/pytest.log 2>&1; s=$?
tail -12 $OUT/pytest.log; [ $s -le 1 ] || exit $s
if [ -x scripts/_spec_probe ]; then
  timeout -k 10 300 scripts/_spec_probe 7070619136 5 > $OUT/spec_probe.json; s2=$?; cat $OUT/spec_probe.json; [ $s2 -eq 0 ] || exit $s2
fi
exit $s
