# bench.py over the BASELINE-shaped configurations on one GPU (one JSON line each):
# configs[0] tiny Llama x 2, configs[1] 125M x 8, the 1.3B x 8 default in the three dtype regimes,
# and larger resident populations. CPU baseline shortened (reported by the default run).
set -u
OUT=gpurun_out/sweep; mkdir -p $OUT
run() {  # name, args
  local name=$1; shift
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 --cpu-baseline-seconds 2 "$@" > $OUT/$name.log 2>&1 \
    || { tail -5 $OUT/$name.log; exit 1; }
  tail -1 $OUT/$name.log > $OUT/$name.json
  python3 -c "import json; d=json.load(open('$OUT/$name.json')); r=d['roofline']; print('$name', d['ms_per_step'], d['value'], r['frac'], r.get('frac_of_stream_ceiling'))"
}
run tiny_k2_f32 --layout tiny_llama --population 2
run gpt2_k8_f32 --layout gpt2_small
run gpt2_k8_mixed --layout gpt2_small --worker-dtype bf16
run 1p3b_k8_f32
run 1p3b_k8_mixed --worker-dtype bf16
run 1p3b_k8_bf16 --worker-dtype bf16 --theta-dtype bf16
run 1p3b_k16_mixed --worker-dtype bf16 --population 16
run 1p3b_k32_mixed --worker-dtype bf16 --population 32
run 1p3b_k3_f32 --population 3
