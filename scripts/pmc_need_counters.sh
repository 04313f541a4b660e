#!/bin/bash
# r5: rocprofv3 counters of the needed-sums population passes (slerp_need_kernel, stats and
# emitting forms) on one roulette-drawn 8 x 7B generation (GRAPH = index into the probe's list; the
# ring of children is index 6 with --ring) — VALU / SALU / wait shares, waves per CU. One counter
# group per pass, never with trace domains, each under its own kill timeout.
set -u
cd "$(dirname "$0")/.."
R=$(pwd); OUT=$R/gpurun_out/${TAG:-r5c}/counters_${GRAPH:-0}
mkdir -p $OUT
pass() {
  local name=$1; shift
  (cd /tmp && export TMPDIR=/tmp && timeout -s KILL 240 rocprofv3 --pmc "$@" --output-format csv \
      -d $OUT/$name -o pmc -- python3 $R/scripts/pop_roulette_probe.py --graphs 6 --ring --rounds 1 --only ${GRAPH:-0} > $OUT/$name.log 2>&1)
  local s=$?; echo "pass $name: status $s"; return $s
}
pass sq SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY \
    SQ_ACTIVE_INST_VALU SQ_INSTS_VALU GRBM_GUI_ACTIVE GRBM_COUNT &&
pass lds SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR
s=$?
python3 scripts/pmc_slerp_counters.py $OUT need > $OUT/summary.json 2> $OUT/summary.err; cat $OUT/summary.json
exit $s
