#!/bin/bash
# Kernel time per step vs batch size (bench.py --no-cpu-baseline), into gpurun_out/$TAG/sweep.txt
set -o pipefail
TAG=${TAG:-sweep}
mkdir -p gpurun_out/$TAG
for env in ${ENVS:-ant_heavenhell}; do
  for B in ${BS:-4096 8192}; do
    timeout -k 10 120 python bench.py --no-cpu-baseline --steps ${STEPS:-100} --env $env --batch $B > gpurun_out/$TAG/$env.$B.json 2>/dev/null || exit 1
    python -c "import json; d=json.load(open('gpurun_out/$TAG/$env.$B.json')); print('$env', $B, d['roofline']['kernel_ms'])" | tee -a gpurun_out/$TAG/sweep.txt
  done
done
