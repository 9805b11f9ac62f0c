#!/bin/bash
# Round 4: per-body wall broadphase (four lanes), two-item cooperative rounds (eight / sixteen
# lanes) -- the GPU suite and each BASELINE config's kernel time (two runs).
OUT=gpurun_out/r4k
mkdir -p $OUT
export TMPDIR=/tmp
python scripts/check_fresh.py || exit 3
fatal() { case $1 in 124|134|137|139) echo "fatal exit $1 in $2"; exit $1;; esac; }
timeout -k 10 900 python -u -m pytest tests -m gpu -v -x --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1; rc=$?; fatal $rc pytest
tail -2 $OUT/pytest_gpu.log; grep -E "FAILED|Error" $OUT/pytest_gpu.log | head -20
[ $rc -ne 0 ] && exit $rc
for r in 1 2; do
for cfg in "ant_heavenhell 65536" "ant_tag 65536" "ant_gather 65536" "ant_heavenhell 32768" "ant_heavenhell 4096" "ant_tag 8192" "ant_gather 16384"; do
  set -- $cfg
  timeout -k 10 120 python bench.py --no-cpu-baseline --steps 200 --env $1 --batch $2 > $OUT/libpob.$1.$2.$r.json 2> $OUT/libpob.$1.$2.$r.err || { tail -5 $OUT/libpob.$1.$2.$r.err; exit 1; }
  python -c "import json; d=json.load(open('$OUT/libpob.$1.$2.$r.json')); print('$1 $2', d['roofline']['kernel_ms'])"
done
done
