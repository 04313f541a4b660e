# The multi-GPU (RCCL) schedules at world size 1 on a one-GPU box: bench --sharded for each
# (mode, broadcast) combination, and at K_local = 1 (the per-rank shape of N = 8).
set -u
R=gpurun_out
port=29511
run() {  # name, bench args...
  local name=$1; shift
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 \
      --master-port $port bench.py --sharded --steps 5 --warmup 2 "$@" > $R/bench_sharded_$name.log 2>&1 \
      || { tail -20 $R/bench_sharded_$name.log; exit 1; }
  port=$((port + 1))
  tail -1 $R/bench_sharded_$name.log
}
run reduce --mode reduce
run exact_theta --mode exact --broadcast theta
run exact_workers --mode exact --broadcast workers
run k1_exact_workers --population 1 --mode exact --broadcast workers
