#!/bin/bash
# A/B of build_variants/*.so against the in-tree libpob.so: HH 65 536 / 4 096, TAG 8 192, GA 16 384
# (interleaved, R rounds), output gpurun_out/$TAG/ab.txt
set -o pipefail
TAG=${TAG:?}
mkdir -p gpurun_out/$TAG
rm -rf gpurun_out/ab
R=${R:-3} BS="${BS:-65536 4096}" ENVS="${ENVS:-ant_heavenhell}" STEPS=${STEPS:-100} bash scripts/ab_bench.sh > gpurun_out/$TAG/ab.txt 2>&1 || { tail gpurun_out/$TAG/ab.txt; exit 1; }
if [ -n "${ENVS2:-}" ]; then
  rm -rf gpurun_out/ab
  R=${R:-3} BS="${BS2}" ENVS="${ENVS2}" STEPS=${STEPS:-100} bash scripts/ab_bench.sh >> gpurun_out/$TAG/ab.txt 2>&1 || { tail gpurun_out/$TAG/ab.txt; exit 1; }
fi
cat gpurun_out/$TAG/ab.txt
