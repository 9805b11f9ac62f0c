#!/bin/bash
# GPU suite + smoke + bench of the in-tree build, then env-switch A/Bs: the sixteen-lane kernel
# at B = 16 384 (HH, TAG), the split launch for the mixed fp16 launch (config 5 per GPU)
set -o pipefail
TAG=r7h bash scripts/gpu_check.sh || exit 1
OUT=gpurun_out/r7h
rm -rf gpurun_out/abenv
VARS="POB_HEXA_MAX_B=0;POB_HEXA_MAX_B=16384" ENVS="ant_heavenhell ant_tag" BS="16384" R=3 bash scripts/ab_env.sh > $OUT/ab_hex16384.txt 2>&1 || exit 1
cat $OUT/ab_hex16384.txt
rm -rf gpurun_out/abenv
VARS="POB_QUAD_SPLIT=0;POB_QUAD_SPLIT=1" ENVS="mixed" BS="32768" EXTRA="--qp-dtype f16" R=3 bash scripts/ab_env.sh > $OUT/ab_mixed_split.txt 2>&1 || exit 1
cat $OUT/ab_mixed_split.txt
