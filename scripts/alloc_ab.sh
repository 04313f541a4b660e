# Does the physical placement of the arenas (default caching allocator vs expandable segments,
# i.e. virtual-memory-mapped 2 MiB granules) change the fused step? Same box, alternating runs.
set -u
for rep in 1 2; do
  for conf in default expandable; do
    if [ $conf = expandable ]; then export PYTORCH_HIP_ALLOC_CONF=expandable_segments:True; else unset PYTORCH_HIP_ALLOC_CONF; fi
    timeout -k 10 300 python bench.py --steps 10 --warmup 3 --cpu-baseline-seconds 0 > gpurun_out/ab_$conf$rep.log 2>&1 || exit 1
    echo "$conf $rep $(tail -1 gpurun_out/ab_$conf$rep.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); r=d["roofline"]; print(r["kernel_ms"], r["stream_ceiling_GBps"], r["device_copy_GBps"])')"
  done
done
