#!/bin/bash
# Verdict r2 item 4: rocprofv3 counters of the speculative SLERP pass against lerp_kernel (and the
# two-pass stats / blend) on the same 7B arenas (scripts/slerp_spec_probe.py --rounds 1). One
# counter group per pass, never with trace domains; each pass under its own kill timeout. The
# derived metrics (gfx94x formulas on ROCm 7.2, MI355X_MICROARCH.md) run last.
set -u
cd "$(dirname "$0")/.."
R=$(pwd); OUT=$R/gpurun_out/${TAG:-r3c}/counters
mkdir -p $OUT
(cd /tmp && export TMPDIR=/tmp && timeout -s KILL 60 rocprofv3 -L > $OUT/avail.txt 2>&1) || true
pass() {
  local name=$1; shift
  (cd /tmp && export TMPDIR=/tmp && timeout -s KILL 120 rocprofv3 --pmc "$@" --output-format csv \
      -d $OUT/$name -o pmc -- python3 $R/scripts/slerp_spec_probe.py --rounds 1 > $OUT/$name.log 2>&1)
  local s=$?; echo "pass $name: status $s"; return $s
}
pass sq SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY \
    SQ_ACTIVE_INST_VALU SQ_INSTS_VALU GRBM_GUI_ACTIVE GRBM_COUNT &&
pass tcc TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum TCC_HIT_sum TCC_MISS_sum &&
pass lds SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR &&
pass membusy MemUnitBusy &&
pass memstall MemUnitStalled &&
pass wrstall WriteUnitStalled
s=$?
python3 scripts/pmc_slerp_counters.py $OUT > $OUT/summary.json 2> $OUT/summary.err; cat $OUT/summary.json
exit $s
