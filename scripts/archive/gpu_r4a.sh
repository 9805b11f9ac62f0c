#!/bin/bash
# Round 4, first GPU pass: the changed GPU tests, the launcher (2 gloo ranks on the box's one
# GPU), the legacy bench line + its PMC profile, the default bench line.
set -o pipefail
OUT=gpurun_out/r4a
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_legacy.py tests/test_gpu_rollout.py tests/test_lib_symbols.py -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { grep -E "^E |FAILED|Error" $OUT/pytest_gpu.log | head -40; exit 1; }
tail -2 $OUT/pytest_gpu.log
timeout -k 10 300 python bench.py --gpus 2 --dist-backend gloo --no-cpu-baseline --steps 50 > $OUT/bench_gpus2_gloo.json 2> $OUT/bench_gpus2_gloo.err || { tail -20 $OUT/bench_gpus2_gloo.err; exit 1; }
cat $OUT/bench_gpus2_gloo.json
timeout -k 10 300 python bench.py --legacy-spring > $OUT/bench_legacy_hh65536.json 2> $OUT/bench_legacy.err || { tail -20 $OUT/bench_legacy.err; exit 1; }
cat $OUT/bench_legacy_hh65536.json
timeout -k 10 300 python bench.py > $OUT/bench_default.json 2> $OUT/bench_default.err || { tail -20 $OUT/bench_default.err; exit 1; }
cat $OUT/bench_default.json
TAG=r4a_legacy_hh65536 ARGS="--legacy-spring" bash scripts/prof_pmc.sh > $OUT/prof_legacy.log 2>&1 || { tail -20 $OUT/prof_legacy.log; exit 1; }
tail -30 $OUT/prof_legacy.log
