#!/bin/bash
# GPU session: full GPU test suite, default bench, gym bench, profile of the headline config.
set -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"
OUT=gpurun_out/r2a
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 240 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc"
tail -3 $OUT/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py > $OUT/bench_default.json 2> $OUT/bench_default.err || exit $?
cat $OUT/bench_default.json
timeout -k 10 200 python bench.py --gym --no-cpu-baseline > $OUT/bench_gym.json 2> $OUT/bench_gym.err || exit $?
cat $OUT/bench_gym.json
