#!/bin/bash
# Round 4: after the mesh diagonal-candidate fix -- the full GPU suite (out-of-range case
# first), then the four-lane kernel's register-budget A/B (4 waves / SIMD with spills vs
# build_variants/quad3w.so at 3 waves / SIMD).  Test failures do not stop the chain; a
# timeout / abort / crash does.
OUT=gpurun_out/r4e
mkdir -p $OUT
export TMPDIR=/tmp
python scripts/check_fresh.py || exit 3
fatal() { case $1 in 124|134|137|139) echo "fatal exit $1 in $2"; exit $1;; esac; }
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1; rc=$?; fatal $rc pytest
tail -2 $OUT/pytest_gpu.log; grep -E "FAILED" $OUT/pytest_gpu.log | head -20
R=3 BS="65536 32768" ENVS="ant_heavenhell ant_tag" timeout -k 10 400 bash scripts/ab_bench.sh > $OUT/ab_quad3w.txt 2>&1; rc=$?; fatal $rc ab
cat $OUT/ab_quad3w.txt
