#!/bin/bash
# Round 4: the mesh (capsule x TriangulatedBox) contact port -- full GPU suite, then bench lines.
set -o pipefail
OUT=gpurun_out/${TAG:-r4b}
mkdir -p $OUT
export TMPDIR=/tmp
python scripts/check_fresh.py || exit 3
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread ${PYTEST_ARGS:-} > $OUT/pytest_gpu.log 2>&1 || { grep -E "^E |FAILED|Error" $OUT/pytest_gpu.log | head -60; exit 1; }
tail -2 $OUT/pytest_gpu.log
for spec in "default:" "hh_4096:--global-batch 4096" "ga_16384:--env ant_gather --global-batch 16384" "tag_8192:--env ant_tag --global-batch 8192" "tag_65536:--env ant_tag" "legacy:--legacy-spring"; do
  name=${spec%%:*}; args=${spec#*:}
  timeout -k 10 200 python bench.py --no-cpu-baseline $args > $OUT/bench_$name.json 2> $OUT/bench_$name.err || { tail -5 $OUT/bench_$name.err; exit 1; }
  python -c "import json; d=json.load(open('$OUT/bench_$name.json')); print('$name', '%.3e' % d['value'], d['roofline']['kernel_ms'])"
done
