#!/bin/bash
# env-switch A/B: the eight-lane kernel's branch-free guards at two waves per SIMD (HH with its
# contact pool, TAG) -- POB_OCT_GACC auto is on only up to one wave per SIMD (B <= 8 192)
set -o pipefail
mkdir -p gpurun_out/r7o
rm -rf gpurun_out/abenv
VARS="POB_OCT_GACC=0;POB_OCT_GACC=1" ENVS="ant_heavenhell ant_tag" BS="12288 16384" R=3 bash scripts/ab_env.sh > gpurun_out/r7o/ab_oct_gacc.txt 2>&1 || exit 1
cat gpurun_out/r7o/ab_oct_gacc.txt
