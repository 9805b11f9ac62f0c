#!/bin/bash
# kernel switch points with the round-6 kernels: the sixteen-lane kernel (default for HH <= 12 288,
# TAG <= 8 192) against the eight-lane one (POB_HEXA_MAX_B=0)
set -o pipefail
mkdir -p gpurun_out/r7k
rm -rf gpurun_out/abenv
VARS="POB_HEXA_MAX_B=0;POB_HEXA_MAX_B=100000" ENVS="ant_heavenhell" BS="8192 12288" R=3 bash scripts/ab_env.sh > gpurun_out/r7k/ab_hh.txt 2>&1 || exit 1
cat gpurun_out/r7k/ab_hh.txt
rm -rf gpurun_out/abenv
VARS="POB_HEXA_MAX_B=0;POB_HEXA_MAX_B=100000" ENVS="ant_tag" BS="6144 8192" R=3 bash scripts/ab_env.sh > gpurun_out/r7k/ab_tag.txt 2>&1 || exit 1
cat gpurun_out/r7k/ab_tag.txt
