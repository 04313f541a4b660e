set -u
R=gpurun_out
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29511 bench.py --sharded --steps 5 --warmup 2 > $R/bench_sharded_reduce.log 2>&1 || { tail -20 $R/bench_sharded_reduce.log; exit 1; }
tail -1 $R/bench_sharded_reduce.log
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29512 bench.py --sharded --mode exact --steps 5 --warmup 2 > $R/bench_sharded_exact.log 2>&1 || { tail -20 $R/bench_sharded_exact.log; exit 1; }
tail -1 $R/bench_sharded_exact.log
timeout -k 10 300 python scripts/placement_probe.py > $R/placement.json 2>&1 || { tail -5 $R/placement.json; exit 1; }
tail -1 $R/placement.json
