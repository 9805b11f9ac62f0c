#!/bin/bash
# GPU suite + smoke + bench of the in-tree build (mixed launch split), then the eight-lane
# kernel's contact pool (build_variants/octpool.so) A/B
set -o pipefail
TAG=r7i bash scripts/gpu_check.sh || exit 1
TAG=r7i BS="16384" ENVS="ant_heavenhell ant_gather" ENVS2="ant_tag" BS2="12288 16384" R=3 bash scripts/gpu_ab.sh
