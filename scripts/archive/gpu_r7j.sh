#!/bin/bash
# GPU suite + smoke + bench of the in-tree build (eight-lane pool for HH), then A/B of the
# four-lane kernel with the post-loop index re-derivation for HH (build_variants/hh_rederive.so)
set -o pipefail
TAG=r7j bash scripts/gpu_check.sh || exit 1
TAG=r7j BS="65536" ENVS="ant_heavenhell" R=3 bash scripts/gpu_ab.sh
