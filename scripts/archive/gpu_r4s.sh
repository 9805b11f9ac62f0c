#!/bin/bash
# Round 4: A/B of the out-of-line face evaluation (build_variants/outline.so, POB_MESH_OUTLINE)
# against the product build at the four-lane batch sizes and the legacy mode.
OUT=gpurun_out/r4s
mkdir -p $OUT
export TMPDIR=/tmp
python scripts/check_fresh.py || exit 3
fatal() { case $1 in 124|134|137|139) echo "fatal exit $1 in $2"; exit $1;; esac; }
rm -rf gpurun_out/ab
R=3 BS="65536 32768" ENVS="ant_heavenhell ant_tag" timeout -k 10 500 bash scripts/ab_bench.sh > $OUT/ab_outline.txt 2>&1; rc=$?; fatal $rc ab
cat $OUT/ab_outline.txt
rm -rf gpurun_out/ab
R=2 BS="65536" ENVS="ant_heavenhell" EXTRA="--legacy-spring" timeout -k 10 300 bash scripts/ab_bench.sh > $OUT/ab_outline_legacy.txt 2>&1; rc=$?; fatal $rc ab2
cat $OUT/ab_outline_legacy.txt
