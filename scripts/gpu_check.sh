#!/bin/bash
# One GPU-box pass: parity tests, then bench lines for the BASELINE.json configs.
# Every GPU step has its own time limit; the chain stops at the first failure.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -m pytest tests -m gpu -x -q -s > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -3 gpurun_out/pytest_gpu.log
timeout -k 10 300 python bench.py > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err || exit 1
cat gpurun_out/bench_default.json
timeout -k 10 200 python bench.py --env mixed --batch 32768 --qp-dtype f16 --no-cpu-baseline > gpurun_out/bench_mixed_f16.json || exit 1
timeout -k 10 200 python bench.py --env mixed --batch 32768 --no-cpu-baseline > gpurun_out/bench_mixed_f32.json || exit 1
timeout -k 10 200 python bench.py --env ant_heavenhell --batch 65536 --qp-dtype f16 --no-cpu-baseline > gpurun_out/bench_hh_f16.json || exit 1
timeout -k 10 200 python bench.py --env ant_heavenhell --batch 4096 --no-cpu-baseline > gpurun_out/bench_hh_4096.json || exit 1
timeout -k 10 200 python bench.py --env ant_gather --batch 16384 --no-cpu-baseline > gpurun_out/bench_ga_16384.json || exit 1
timeout -k 10 200 python bench.py --env ant_tag --batch 65536 --no-cpu-baseline > gpurun_out/bench_tag_65536.json || exit 1
timeout -k 10 200 python bench.py --env ant --batch 65536 --no-cpu-baseline > gpurun_out/bench_ant_65536.json || exit 1
for f in gpurun_out/bench_*.json; do python -c "import json,sys; d=json.load(open('$f')); print('$f', d['value'], d['ms_per_step'], d['roofline']['frac'])"; done
