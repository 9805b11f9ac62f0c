#!/bin/bash
# Round 4: zero-distance wall contacts kept out of the range guards -- the GPU suite, then A/B
# of the wave walk (libpob), the per-lane walk with the same fix (build_variants/seqx.so) and
# the previous build (build_variants/seqwalk.so), with the automatic guard policy and with the
# branch guards forced (POB_HEX_GACC = POB_OCT_GACC = 0).
OUT=gpurun_out/r4h
mkdir -p $OUT
export TMPDIR=/tmp
python scripts/check_fresh.py || exit 3
fatal() { case $1 in 124|134|137|139) echo "fatal exit $1 in $2"; exit $1;; esac; }
timeout -k 10 900 python -u -m pytest tests -m gpu -v -x --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1; rc=$?; fatal $rc pytest
tail -2 $OUT/pytest_gpu.log; grep -E "FAILED|Error" $OUT/pytest_gpu.log | head -20
[ $rc -ne 0 ] && exit $rc
rm -rf gpurun_out/ab
R=2 BS="65536 8192 4096" ENVS="ant_heavenhell ant_tag" timeout -k 10 600 bash scripts/ab_bench.sh > $OUT/ab1.txt 2>&1; rc=$?; fatal $rc ab1
cat $OUT/ab1.txt
rm -rf gpurun_out/ab
POB_HEX_GACC=0 POB_OCT_GACC=0 R=2 BS="8192 4096" ENVS="ant_heavenhell ant_tag" timeout -k 10 400 bash scripts/ab_bench.sh > $OUT/ab_nogacc.txt 2>&1; rc=$?; fatal $rc ab2
echo "== branch guards forced"; cat $OUT/ab_nogacc.txt
