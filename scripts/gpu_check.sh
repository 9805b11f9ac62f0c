#!/bin/bash
# One GPU pass of the current build: the GPU test suite, smoke(), and the default bench line,
# each step under its own time limit, stopping at the first failure.  Output in
# gpurun_out/$TAG/ (copy what is to be kept into profiles/).
#   TAG=r7a bash scripts/gpu_check.sh [extra bench.py args for the bench step]
set -o pipefail
TAG=${TAG:?}
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 \
  || { tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -2 $OUT/pytest_gpu.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -20 $OUT/smoke.log; exit 1; }
timeout -k 10 300 python -u bench.py "$@" > $OUT/bench_default.json 2> $OUT/bench_default.err || { tail -20 $OUT/bench_default.err; exit 1; }
cat $OUT/bench_default.json
