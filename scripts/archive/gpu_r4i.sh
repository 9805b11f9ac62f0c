#!/bin/bash
# Round 4: the four-lane kernel back on the per-lane walk with face-level contact masks --
# the GPU suite; A/B against wall-level masks (build_variants/qwallhit.so); the small-batch
# breakdown of the eight- / sixteen-lane kernels (no face walk, no walls: build_variants_t/).
OUT=gpurun_out/r4i
mkdir -p $OUT
export TMPDIR=/tmp
python scripts/check_fresh.py || exit 3
fatal() { case $1 in 124|134|137|139) echo "fatal exit $1 in $2"; exit $1;; esac; }
timeout -k 10 900 python -u -m pytest tests -m gpu -v -x --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1; rc=$?; fatal $rc pytest
tail -2 $OUT/pytest_gpu.log; grep -E "FAILED|Error" $OUT/pytest_gpu.log | head -20
[ $rc -ne 0 ] && exit $rc
rm -rf gpurun_out/ab
R=2 BS="65536 32768" ENVS="ant_heavenhell ant_tag" timeout -k 10 400 bash scripts/ab_bench.sh > $OUT/ab_quad.txt 2>&1; rc=$?; fatal $rc ab
cat $OUT/ab_quad.txt
for cfg in "ant_heavenhell 4096" "ant_tag 8192" "ant_gather 16384"; do
  set -- $cfg
  for lib in po-brax_amd/po_brax_amd/libpob.so build_variants_t/nowalk.so build_variants_t/nowalls.so; do
    tag=$(basename $lib .so)
    POB_LIB=$PWD/$lib timeout -k 10 120 python bench.py --no-cpu-baseline --steps 200 --env $1 --batch $2 > $OUT/$tag.$1.$2.json 2> $OUT/$tag.$1.$2.err || { tail -5 $OUT/$tag.$1.$2.err; exit 1; }
    python -c "import json; d=json.load(open('$OUT/$tag.$1.$2.json')); print('$1 $2 $tag', d['roofline']['kernel_ms'])"
  done
done
