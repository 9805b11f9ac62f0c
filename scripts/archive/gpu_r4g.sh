#!/bin/bash
# Round 4: the wave-cooperative wall walk -- the full GPU suite, then A/B against the per-lane
# walk (build_variants/seqwalk.so, the previous build) over the BASELINE batch sizes.
OUT=gpurun_out/r4g
mkdir -p $OUT
export TMPDIR=/tmp
python scripts/check_fresh.py || exit 3
fatal() { case $1 in 124|134|137|139) echo "fatal exit $1 in $2"; exit $1;; esac; }
timeout -k 10 900 python -u -m pytest tests -m gpu -v -x --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1; rc=$?; fatal $rc pytest
tail -2 $OUT/pytest_gpu.log; grep -E "FAILED|Error" $OUT/pytest_gpu.log | head -20
[ $rc -ne 0 ] && exit $rc
R=2 BS="65536 8192 4096" ENVS="ant_heavenhell ant_tag" timeout -k 10 500 bash scripts/ab_bench.sh > $OUT/ab1.txt 2>&1; rc=$?; fatal $rc ab1
cat $OUT/ab1.txt
rm -f gpurun_out/ab/*.json
R=2 BS="16384" ENVS="ant_gather" timeout -k 10 200 bash scripts/ab_bench.sh > $OUT/ab2.txt 2>&1; rc=$?; fatal $rc ab2
cat $OUT/ab2.txt
