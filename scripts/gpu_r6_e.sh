#!/bin/bash
# r6: the multi-GPU line's code path at world size 1 over RCCL on the final library, full size
# (bench.py --gpus 1 --sharded: the sharded schedule, every extra, parity), capped line + sidecar.
set -o pipefail
O=gpurun_out/r6e
mkdir -p $O
timeout -k 10 900 python3 -u bench.py --gpus 1 --sharded --detail-out $O/sharded_world1_detail.json \
    > $O/sharded_world1.json 2> $O/sharded_world1.err || { tail -30 $O/sharded_world1.err; exit 1; }
wc -c $O/sharded_world1.json
cut -c1-1500 $O/sharded_world1.json
echo done
