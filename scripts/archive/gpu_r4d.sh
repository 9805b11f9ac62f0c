#!/bin/bash
# Round 4: debug the out-of-range parity case, run the rest of the GPU suite, A/B the four-lane
# kernel's register budget (4 waves / SIMD with spills vs 3 waves / SIMD).  Test failures do
# not stop the chain; a timeout / abort / crash does.
OUT=gpurun_out/r4d
mkdir -p $OUT
export TMPDIR=/tmp
python scripts/check_fresh.py || exit 3
fatal() { case $1 in 124|134|137|139) echo "fatal exit $1 in $2"; exit $1;; esac; }
for c in "8 70 1" "8 70 0" "16 70 1" "4 70 none"; do
  timeout -k 10 200 python scripts/debug_oor.py $c > $OUT/oor_${c// /_}.txt 2>&1; rc=$?; fatal $rc "oor $c"
  echo "== $c rc=$rc"; head -8 $OUT/oor_${c// /_}.txt
done
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread --deselect "tests/test_gpu_headline_parity.py::test_out_of_range_inputs_take_exact_fallbacks" > $OUT/pytest_gpu.log 2>&1; rc=$?; fatal $rc pytest
tail -2 $OUT/pytest_gpu.log; grep -E "FAILED" $OUT/pytest_gpu.log | head -20
R=3 BS="65536 32768" ENVS="ant_heavenhell ant_tag" timeout -k 10 400 bash scripts/ab_bench.sh > $OUT/ab_quad3w.txt 2>&1; rc=$?; fatal $rc ab
cat $OUT/ab_quad3w.txt
