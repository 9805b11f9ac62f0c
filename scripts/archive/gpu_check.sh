#!/bin/bash
# One GPU-box pass: parity tests, then bench lines for the BASELINE.json configs (and the
# gym path), all into gpurun_out/$TAG/.  Every GPU step has its own time limit; the chain
# stops at the first failure.   TAG=r2h bash scripts/gpu_check.sh [--no-tests]
set -o pipefail
TAG=${TAG:-check}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
if [ "${1:-}" != "--no-tests" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { grep -E "^E |FAILED" $OUT/pytest_gpu.log | head -30; exit 1; }
  tail -2 $OUT/pytest_gpu.log
fi
timeout -k 10 300 python bench.py > $OUT/bench_default.json 2> $OUT/bench_default.err || exit 1
run() {  # name, bench args...
  local name=$1; shift
  timeout -k 10 200 python bench.py --no-cpu-baseline "$@" > $OUT/bench_$name.json 2> $OUT/bench_$name.err || exit 1
}
run hh_4096 --batch 4096 &&
run tag_8192 --env ant_tag --batch 8192 &&
run ga_16384 --env ant_gather --batch 16384 &&
run tag_65536 --env ant_tag --batch 65536 &&
run mixed_f16_32768 --env mixed --qp-dtype f16 --batch 32768 &&
run mixed_f32_32768 --env mixed --batch 32768 &&
run hh_f16 --qp-dtype f16 &&
run ant_65536 --env ant --batch 65536 &&
run gym_hh --gym &&
run hh_steady --steps 1000 --warmup 50 || exit 1
for f in $OUT/bench_*.json; do python -c "import json,sys; d=json.load(open('$f')); r=d['roofline']; print('$f', d['value'], d['ms_per_step'], r['kernel_ms'], r['frac'])"; done
