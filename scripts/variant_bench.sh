#!/bin/bash
# Bench the default libpob.so (each step kernel via POB_STEP_LANES) against variant
# builds in build_variants/ (same workload).
set -o pipefail
shopt -s nullglob
mkdir -p gpurun_out/variants
run() {  # tag lib lanes B
  POB_STEP_LANES=$3 POB_LIB=$PWD/$2 timeout -k 10 200 python bench.py --no-cpu-baseline --steps 200 --batch $4 > gpurun_out/variants/$1.$4.json 2>/dev/null || exit 1
  python -c "import json; d=json.load(open('gpurun_out/variants/$1.$4.json')); print('$1', $4, d['value'], d['roofline']['kernel_ms'])"
}
for B in 65536 4096; do
  run pair po-brax_amd/po_brax_amd/libpob.so 2 $B
  run quad po-brax_amd/po_brax_amd/libpob.so 4 $B
  for lib in build_variants/*.so; do run $(basename $lib .so) $lib 4 $B; done
done
