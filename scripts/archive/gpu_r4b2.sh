#!/bin/bash
# debug the out-of-range parity case, then the rest of the GPU suite
set -o pipefail
OUT=gpurun_out/r4b2
mkdir -p $OUT
export TMPDIR=/tmp
for c in "8 70 1" "8 70 0" "16 70 1" "4 70 none"; do
  timeout -k 10 200 python scripts/debug_oor.py $c > $OUT/oor_${c// /_}.txt 2>&1 || { tail -5 $OUT/oor_${c// /_}.txt; exit 1; }
  echo "== $c"; head -12 $OUT/oor_${c// /_}.txt
done
timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread --deselect "tests/test_gpu_headline_parity.py::test_out_of_range_inputs_take_exact_fallbacks" > $OUT/pytest_gpu.log 2>&1; tail -3 $OUT/pytest_gpu.log; grep -E "FAILED" $OUT/pytest_gpu.log | head -20
