#!/bin/bash
# Round 4, final tree: the GPU suite, smoke and the default bench line on the committed build.
set -o pipefail
OUT=gpurun_out/r4u
mkdir -p $OUT
export TMPDIR=/tmp
python scripts/check_fresh.py || exit 3
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -20 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -20 $OUT/smoke.log; exit 1; }
tail -2 $OUT/smoke.log
timeout -k 10 300 python bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail -10 $OUT/bench.err; exit 1; }
python -c "import json; d=json.load(open('$OUT/bench.json')); print('%.4e' % d['value'], d['roofline']['kernel_ms'], d['cpu_baseline'])"
