set -o pipefail
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -3 gpurun_out/pytest_gpu.log
timeout -k 10 300 python scripts/bench_generation.py --layout gpt2_small --json gpurun_out/gen_125m.json > gpurun_out/gen_125m.log 2>&1 && tail -3 gpurun_out/gen_125m.log
timeout -k 10 300 python scripts/bench_generation.py --layout gpt_1p3b --json gpurun_out/gen_1p3b.json > gpurun_out/gen_1p3b.log 2>&1 && tail -3 gpurun_out/gen_1p3b.log
