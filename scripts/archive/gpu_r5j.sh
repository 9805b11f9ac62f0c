#!/bin/bash
# counters of the four-lane kernel variants at HH B = 65 536 (build_variants/*.so via POB_LIB)
set -o pipefail
for v in nowalk wave_inl lane_inl; do
  POB_LIB=$PWD/build_variants/$v.so TAG=r5j_$v SETS="SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_INSTS_SALU SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VMEM;GRBM_GUI_ACTIVE;FETCH_SIZE;WRITE_SIZE" \
    bash scripts/prof_pmc.sh > gpurun_out/prof_r5j_$v.txt 2>&1 || { tail -5 gpurun_out/prof_r5j_$v.txt; exit 1; }
  grep -E "k_step_quad|SQ_INSTS_VALU:|SQ_WAVE_CYCLES|SQ_WAIT_ANY|HBM bytes" profiles/r5j_${v}_summary.md
done
