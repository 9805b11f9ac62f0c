# PMC profiles of the small-batch kernels after the round-3 changes
set -o pipefail
TAG=r3o_hh4096 ARGS="--global-batch 4096" bash scripts/prof_pmc.sh > gpurun_out/pmc_r3o_1.txt 2>&1 || { tail -5 gpurun_out/pmc_r3o_1.txt; exit 1; }
TAG=r3o_tag8192 ARGS="--env ant_tag --global-batch 8192" bash scripts/prof_pmc.sh > gpurun_out/pmc_r3o_2.txt 2>&1 || { tail -5 gpurun_out/pmc_r3o_2.txt; exit 1; }
TAG=r3o_hh8192 ARGS="--global-batch 8192" bash scripts/prof_pmc.sh > gpurun_out/pmc_r3o_3.txt 2>&1 || { tail -5 gpurun_out/pmc_r3o_3.txt; exit 1; }
echo ok
