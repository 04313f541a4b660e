#!/bin/bash
# One GPU session: smoke, GPU tests, a short bench, and a rocprofv3 kernel-trace summary.
# Every GPU step has its own time limit; the script stops at the first fault/abort/timeout.
set -u
cd "$(dirname "$0")/.."
OUT=gpurun_out
mkdir -p $OUT
stop_if_fatal() {  # $1 = exit status of the previous GPU step
  case "$1" in
    0|1) return 0 ;;                 # ok / ordinary test failure
    *) echo "fatal status $1 - stopping"; exit "$1" ;;
  esac
}
echo "== smoke"; timeout -k 10 300 python __graft_entry__.py smoke > $OUT/smoke.log 2>&1; s=$?; tail -3 $OUT/smoke.log; stop_if_fatal $s
echo "== pytest -m gpu"; timeout -k 10 900 python -m pytest tests -q -m gpu ${PYTEST_ARGS:-} > $OUT/pytest_gpu.log 2>&1; s=$?; tail -15 $OUT/pytest_gpu.log; stop_if_fatal $s
echo "== bench"; timeout -k 10 600 python bench.py ${BENCH_ARGS:-} > $OUT/bench.log 2>&1; s=$?; tail -3 $OUT/bench.log; stop_if_fatal $s
if [ "${PROFILE:-1}" = "1" ]; then
  echo "== rocprofv3 kernel trace"
  R=$(pwd)
  (cd /tmp && export TMPDIR=/tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv \
      -d $R/$OUT/prof -o bench -- python3 $R/bench.py ${BENCH_ARGS:-} \
      > $R/$OUT/prof.log 2>&1); s=$?; tail -3 $OUT/prof.log; stop_if_fatal $s   # the bench command itself
  find $OUT/prof -name "*stats*" | head
fi
echo "== done"
