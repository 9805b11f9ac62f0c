#!/bin/bash
# Kernel time per step of library variants (LIBS: in-tree libpob.so = "base", or
# build_variants/NAME.so) x staged state load on / off (POB_STAGE=0: per-lane loads), per
# env and batch, into gpurun_out/$TAG/sweep.txt.
set -o pipefail
TAG=${TAG:-stage}
OUT=gpurun_out/$TAG
mkdir -p $OUT
for env in ${ENVS:-ant_heavenhell ant_gather}; do
  for B in ${BS:-4096 16384 32768 65536}; do
    for lib in ${LIBS:-base}; do
      for st in ${STAGES:-1 0}; do
        if [ $lib = base ]; then lp=""; else lp=$PWD/build_variants/$lib.so; fi
        f=$OUT/$env.$B.$lib.s$st.json
        POB_LIB=${lp:-$PWD/po-brax_amd/po_brax_amd/libpob.so} POB_STAGE=$st timeout -k 10 120 python bench.py --no-cpu-baseline \
          --steps ${STEPS:-200} --env $env --batch $B > $f 2> $OUT/$env.$B.$lib.s$st.err || exit 1
        python -c "import json; d=json.load(open('$f')); r=d['roofline']; print('$env', $B, '$lib', 'stage=$st', r['kernel_ms'], r.get('kernel'))" | tee -a $OUT/sweep.txt
      done
    done
  done
done
