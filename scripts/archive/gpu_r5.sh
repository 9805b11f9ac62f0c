#!/bin/bash
# Round 5 GPU pass: freshness check, the GPU suite, smoke, and bench lines for the BASELINE
# configs (one process each, own time limits; the chain stops at the first failure).
#   OUT=gpurun_out/r5a [SKIP_TESTS=1] [BENCH="..."] bash scripts/gpu_r5.sh
set -o pipefail
OUT=${OUT:?}
mkdir -p $OUT
export TMPDIR=/tmp
python scripts/check_fresh.py || exit 3
if [ -z "${SKIP_TESTS:-}" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread ${PYTEST_K:-} > $OUT/pytest_gpu.log 2>&1 || { tail -30 $OUT/pytest_gpu.log; exit 1; }
  tail -1 $OUT/pytest_gpu.log
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -20 $OUT/smoke.log; exit 1; }
  tail -4 $OUT/smoke.log
fi
if [ -z "${SKIP_DEFAULT_BENCH:-}" ]; then
  timeout -k 10 300 python bench.py > $OUT/bench_default.json 2> $OUT/bench_default.err || { tail -10 $OUT/bench_default.err; exit 1; }
  python -c "import json; d=json.load(open('$OUT/bench_default.json')); print('default', '%.4e' % d['value'], d['roofline']['kernel_ms'], d['roofline']['frac'])"
fi
i=0
IFS=';' read -ra CFG <<< "${BENCH:---env ant_heavenhell --global-batch 4096;--env ant_tag --global-batch 8192;--env ant_gather --global-batch 16384;--env ant_tag;--env mixed --qp-dtype f16 --global-batch 32768}"
for c in "${CFG[@]}"; do
  i=$((i + 1))
  timeout -k 10 180 python bench.py --no-cpu-baseline --steps ${STEPS:-200} $c > $OUT/bench_$i.json 2> $OUT/bench_$i.err || { tail -10 $OUT/bench_$i.err; exit 1; }
  python -c "import json; d=json.load(open('$OUT/bench_$i.json')); print('$c', '%.4e' % d['value'], d['roofline']['kernel_ms'])"
done
