#!/bin/bash
# r4: rocprofv3 counters of BASELINE configs[4]'s population passes (the Gram pass, the member-major
# blend, the co-located speculative pass) over scripts/pop_slerp_probe.py --rounds 1: is the Gram
# pass VALU- or memory-bound? One counter group per pass, never with trace domains, each pass under
# its own kill timeout; the summary (scripts/pmc_slerp_counters.py ... pop) runs last.
set -u
cd "$(dirname "$0")/.."
R=$(pwd); OUT=$R/gpurun_out/${TAG:-r4popc}/counters
mkdir -p $OUT
PAIRS=${PAIRS:-probe}
pass() {
  local name=$1; shift
  (cd /tmp && export TMPDIR=/tmp && timeout -s KILL 180 rocprofv3 --pmc "$@" --output-format csv \
      -d $OUT/$name -o pmc -- python3 $R/scripts/pop_slerp_probe.py --rounds 1 --pairs $PAIRS > $OUT/$name.log 2>&1)
  local s=$?; echo "pass $name: status $s"; return $s
}
pass sq SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY \
    SQ_ACTIVE_INST_VALU SQ_INSTS_VALU GRBM_GUI_ACTIVE GRBM_COUNT &&
pass lds SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR
s=$?
python3 scripts/pmc_slerp_counters.py $OUT pop > $OUT/summary.json 2> $OUT/summary.err; cat $OUT/summary.json
exit $s
