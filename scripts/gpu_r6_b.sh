#!/bin/bash
# r6 second call: GPU suite on the lerp nt-store build, the configs[1] joint placement probe, the
# resident populations' output-placement probes (EDT-LM 1.3B, SLERP 7B).
set -o pipefail
O=gpurun_out/r6b
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > $O/pytest_gpu.log 2>&1 \
    || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
JOINT_ONLY=1 timeout -k 10 300 python3 -u scripts/config1_probe.py > $O/config1_joint.jsonl 2> $O/config1_joint.err || { tail -20 $O/config1_joint.err; exit 1; }
cut -c1-300 $O/config1_joint.jsonl
timeout -k 10 300 python3 -u scripts/population_placement_probe.py lm > $O/pop_place_lm.jsonl 2> $O/pop_place_lm.err || { tail -20 $O/pop_place_lm.err; exit 1; }
cat $O/pop_place_lm.jsonl
timeout -k 10 400 python3 -u scripts/population_placement_probe.py slerp > $O/pop_place_slerp.jsonl 2> $O/pop_place_slerp.err || { tail -20 $O/pop_place_slerp.err; exit 1; }
cat $O/pop_place_slerp.jsonl
echo done
