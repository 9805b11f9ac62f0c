#!/bin/bash
# Quick GPU pass: the -m gpu suite, then the headline + small-batch bench lines into
# gpurun_out/$TAG/.  Each step has its own time limit; the chain stops at the first failure.
set -o pipefail
TAG=${TAG:-quick}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { grep -E "^E |FAILED|Error" $OUT/pytest_gpu.log | head -40; exit 1; }
tail -2 $OUT/pytest_gpu.log
for spec in "default:" "hh_4096:--batch 4096" "ga_16384:--env ant_gather --batch 16384" "tag_8192:--env ant_tag --batch 8192"; do
  name=${spec%%:*}; args=${spec#*:}
  timeout -k 10 200 python bench.py --no-cpu-baseline $args > $OUT/bench_$name.json 2> $OUT/bench_$name.err || exit 1
  python -c "import json; d=json.load(open('$OUT/bench_$name.json')); print('$name', '%.3e' % d['value'], d['roofline']['kernel_ms'])"
done
