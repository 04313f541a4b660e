# rocprofv3 kernel-trace summaries of the secondary paths: the resident generations (population
# kernels) and the single-pair merges (pair merge, lerp, SLERP two-pass / speculative).
set -u
R=$(pwd); OUT=$R/gpurun_out/prof2
mkdir -p $OUT
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv \
    -d $OUT/gen -o gen -- python3 $R/scripts/bench_generation.py --layout gpt_1p3b --members lineage \
    > $OUT/gen.log 2>&1) || { tail -5 $OUT/gen.log; exit 1; }
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv \
    -d $OUT/ops -o ops -- python3 $R/scripts/bench_ops.py --ops pair,slerp \
    > $OUT/ops.log 2>&1) || { tail -5 $OUT/ops.log; exit 1; }
tail -1 $OUT/gen.log; tail -1 $OUT/ops.log
