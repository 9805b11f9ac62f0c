# PMC passes of the four-lane and eight-lane kernels at one wave per SIMD (HH B = 16 384)
set -o pipefail
S1="SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SALU"
S2="SQ_INSTS_SMEM SQ_INSTS_LDS SQ_INSTS_VMEM SQ_INSTS_BRANCH SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_SALU SQ_WAIT_INST_LDS"
export SETS="$S1;$S2"
POB_HEXA_MAX_B=0 POB_OCTET_MAX_B=0 TAG=x_quad_hh16384 ARGS="--global-batch 16384" bash scripts/prof_pmc.sh > gpurun_out/x_quad.txt 2>&1 || exit 1
POB_HEXA_MAX_B=0 TAG=x_oct_hh16384 ARGS="--global-batch 16384" bash scripts/prof_pmc.sh > gpurun_out/x_oct.txt 2>&1 || exit 1
POB_HEXA_MAX_B=0 TAG=x_oct_hh8192 ARGS="--global-batch 8192" bash scripts/prof_pmc.sh > gpurun_out/x_oct8.txt 2>&1 || exit 1
echo done
