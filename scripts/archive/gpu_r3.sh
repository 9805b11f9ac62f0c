#!/bin/bash
# Round-3 GPU pass: selected (or all) -m gpu tests, then bench lines into gpurun_out/$TAG/.
# Every GPU step has its own time limit; the chain stops at the first failure.
#   TAG=r3b K="gym_graph or eval_wrapper" bash scripts/gpu_r3.sh
set -o pipefail
TAG=${TAG:-r3}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
if [ -n "${K:-}" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread -k "$K" > $OUT/pytest_gpu.log 2>&1 || { grep -E "^E |FAILED|Error" $OUT/pytest_gpu.log | head -40; exit 1; }
  tail -1 $OUT/pytest_gpu.log
fi
run() {  # name, bench args...
  local name=$1; shift
  timeout -k 10 200 python bench.py --no-cpu-baseline "$@" > $OUT/bench_$name.json 2> $OUT/bench_$name.err || { tail -5 $OUT/bench_$name.err; exit 1; }
  python -c "import json; d=json.load(open('$OUT/bench_$name.json')); print('$name', '%.3e' % d['value'], d['ms_per_step'], d['roofline']['kernel_ms'], d['roofline']['frac'])"
}
for spec in ${BENCHES:-default:}; do
  name=${spec%%:*}; args=${spec#*:}
  run $name ${args//,/ } || exit 1
done
