#!/bin/bash
# Kernel time per step of the quad / octet / hexa step kernels at the batch sizes where the
# launch switches between them (POB_OCTET_MAX_B / POB_HEXA_MAX_B force a kernel), into
# gpurun_out/$TAG/sweep.txt.  Each bench run has its own time limit; the chain stops at the
# first failure.
set -o pipefail
TAG=${TAG:-thr}
OUT=gpurun_out/$TAG
mkdir -p $OUT
for env in ${ENVS:-ant_heavenhell ant_gather ant_tag}; do
  for B in ${BS:-8192 16384 32768}; do
    for v in quad oct hex; do
      case $v in
        quad) ev="POB_OCTET_MAX_B=0 POB_HEXA_MAX_B=0" ;;
        oct) ev="POB_OCTET_MAX_B=1000000 POB_HEXA_MAX_B=0" ;;
        hex) ev="POB_OCTET_MAX_B=0 POB_HEXA_MAX_B=1000000" ;;
      esac
      f=$OUT/$env.$B.$v.json
      env $ev timeout -k 10 120 python bench.py --no-cpu-baseline --steps ${STEPS:-200} --env $env --batch $B > $f 2> $OUT/$env.$B.$v.err || exit 1
      python -c "import json; d=json.load(open('$f')); r=d['roofline']; print('$env', $B, '$v', r['kernel_ms'], r.get('kernel'))" | tee -a $OUT/sweep.txt
    done
  done
done
