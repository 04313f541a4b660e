#!/bin/bash
# Round 4: the whole GPU suite, then the SLERP probe (far parents) once under rocprofv3
# --kernel-trace (the run that crashed at exit in r3 with the hold form).
set -u
cd "$(dirname "$0")/.."
R=$(pwd); OUT=$R/gpurun_out/${TAG:-r4check}
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest ${TESTS:-tests} -m gpu --maxfail=10 -q --timeout 300 --timeout-method thread -p no:cacheprovider \
    > $OUT/pytest_gpu.log 2>&1; s=$?
tail -5 $OUT/pytest_gpu.log; [ $s -eq 0 ] || exit $s
if [ "${PROBE:-1}" = 1 ]; then
  (cd /tmp && export TMPDIR=/tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv \
      -d $OUT/kt -o probe -- python3 $R/scripts/slerp_spec_probe.py --rounds 3 --far > $OUT/kt.log 2>&1); s=$?
  echo "probe under rocprofv3 exit $s"; tail -3 $OUT/kt.log; [ $s -eq 0 ] || exit $s
fi
echo done
