#!/bin/bash
# Bench the default libpob.so against variant builds in build_variants/ (same workload).
set -o pipefail
mkdir -p gpurun_out/variants
for lib in po-brax_amd/po_brax_amd/libpob.so build_variants/*.so; do
  tag=$(basename $lib .so)
  for B in 65536 4096; do
    POB_LIB=$PWD/$lib timeout -k 10 200 python bench.py --no-cpu-baseline --steps 200 --batch $B > gpurun_out/variants/$tag.$B.json 2>/dev/null || exit 1
    python -c "import json; d=json.load(open('gpurun_out/variants/$tag.$B.json')); print('$tag', $B, d['value'], d['roofline']['kernel_ms'])"
  done
done
