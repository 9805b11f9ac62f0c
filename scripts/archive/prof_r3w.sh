set -o pipefail
TAG=r3w_hh65536 ARGS="" bash scripts/prof_pmc.sh > gpurun_out/r3w_1.log 2>&1 || exit 1
TAG=r3w_hh4096 ARGS="--global-batch 4096" bash scripts/prof_pmc.sh > gpurun_out/r3w_2.log 2>&1 || exit 1
TAG=r3w_tag8192 ARGS="--env ant_tag --global-batch 8192" bash scripts/prof_pmc.sh > gpurun_out/r3w_3.log 2>&1 || exit 1
TAG=r3w_ga16384 ARGS="--env ant_gather --global-batch 16384" bash scripts/prof_pmc.sh > gpurun_out/r3w_4.log 2>&1 || exit 1
echo done
