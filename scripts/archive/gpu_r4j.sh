#!/bin/bash
# Round 4: mesh_face with the shared end-point pass -- the GPU suite; each config with the
# product build and the timing builds (build_variants_t/: walk compiled in but never run, no walls).
OUT=gpurun_out/r4j
mkdir -p $OUT
export TMPDIR=/tmp
python scripts/check_fresh.py || exit 3
fatal() { case $1 in 124|134|137|139) echo "fatal exit $1 in $2"; exit $1;; esac; }
timeout -k 10 900 python -u -m pytest tests -m gpu -v -x --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1; rc=$?; fatal $rc pytest
tail -2 $OUT/pytest_gpu.log; grep -E "FAILED|Error" $OUT/pytest_gpu.log | head -20
[ $rc -ne 0 ] && exit $rc
for r in 1 2; do
for cfg in "ant_heavenhell 65536" "ant_tag 65536" "ant_heavenhell 4096" "ant_tag 8192" "ant_gather 16384"; do
  set -- $cfg
  libs="po-brax_amd/po_brax_amd/libpob.so build_variants_t/nowalls.so"
  [ $2 = 65536 ] && libs="$libs build_variants_t/walkdead.so"
  for lib in $libs; do
    tag=$(basename $lib .so)
    POB_LIB=$PWD/$lib timeout -k 10 120 python bench.py --no-cpu-baseline --steps 200 --env $1 --batch $2 > $OUT/$tag.$1.$2.$r.json 2> $OUT/$tag.$1.$2.$r.err || { tail -5 $OUT/$tag.$1.$2.$r.err; exit 1; }
    python -c "import json; d=json.load(open('$OUT/$tag.$1.$2.$r.json')); print('$1 $2 $tag', d['roofline']['kernel_ms'])"
  done
done
done
