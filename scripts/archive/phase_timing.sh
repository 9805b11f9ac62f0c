#!/bin/bash
# Per-phase wave timings (s_memtime ticks) of the step kernel: builds with -DPOB_EXP_TIMING
# (see step_quad_body) print one line per launch for three blocks.  Run on the GPU box:
#   bash scripts/phase_timing.sh   (expects build_variants/libpob_timing*.so)
set -o pipefail
mkdir -p gpurun_out
for lib in build_variants/libpob_timing*.so; do
  v=$(basename $lib .so)
  for B in 65536 4096; do
    POB_LIB=$PWD/$lib timeout -k 10 120 python bench.py --no-cpu-baseline --steps 2 --warmup 1 --batch $B \
        > gpurun_out/ts_${v}_$B.out 2> gpurun_out/ts_${v}_$B.err || exit 1
    echo "== $v B=$B"; grep POBTS gpurun_out/ts_${v}_$B.out | tail -6 || true
  done
done
