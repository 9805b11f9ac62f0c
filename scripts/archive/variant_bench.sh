#!/bin/bash
# Bench the default libpob.so against variant builds in build_variants/ (same workload).
set -o pipefail
shopt -s nullglob
mkdir -p gpurun_out/variants
run() {  # tag lib B
  POB_LIB=$PWD/$2 timeout -k 10 200 python bench.py --no-cpu-baseline --steps 200 --batch $3 > gpurun_out/variants/$1.$3.json 2>/dev/null || exit 1
  python -c "import json; d=json.load(open('gpurun_out/variants/$1.$3.json')); print('$1', $3, d['value'], d['roofline']['kernel_ms'])"
}
for B in ${BS:-65536 4096}; do
  run default po-brax_amd/po_brax_amd/libpob.so $B
  for lib in build_variants/*.so; do run $(basename $lib .so) $lib $B; done
done
