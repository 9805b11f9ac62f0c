#!/bin/bash
# A/B: the four-lane fast launch's walk with branch-free guards (build_variants/quad_walk_gacc.so)
# at HH / TAG 65 536; the eight-lane kernel at B = 32 768 (POB_OCTET_MAX_B) for HH and TAG
set -o pipefail
TAG=r7m BS="65536" ENVS="ant_heavenhell ant_tag" R=3 bash scripts/gpu_ab.sh || exit 1
rm -rf gpurun_out/abenv
VARS="POB_OCTET_MAX_B=16384;POB_OCTET_MAX_B=32768" ENVS="ant_heavenhell ant_tag" BS="32768" R=3 bash scripts/ab_env.sh > gpurun_out/r7m/ab_oct32768.txt 2>&1 || exit 1
cat gpurun_out/r7m/ab_oct32768.txt
