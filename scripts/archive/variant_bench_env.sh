#!/bin/bash
# Bench the default libpob.so against build_variants/*.so on one env / batch:
#   bash scripts/variant_bench_env.sh ENV B [ENV B ...]
set -o pipefail
shopt -s nullglob
mkdir -p gpurun_out/variants
while [ $# -ge 2 ]; do
  ENV=$1; B=$2; shift 2
  for lib in po-brax_amd/po_brax_amd/libpob.so build_variants/*.so; do
    tag=$(basename $lib .so)
    POB_LIB=$PWD/$lib timeout -k 10 200 python bench.py --no-cpu-baseline --steps 200 --env $ENV --batch $B \
        > gpurun_out/variants/$tag.$ENV.$B.json 2>/dev/null || exit 1
    python -c "import json; d=json.load(open('gpurun_out/variants/$tag.$ENV.$B.json')); print('$tag', '$ENV', $B, d['value'], d['roofline']['kernel_ms'])"
  done
done
