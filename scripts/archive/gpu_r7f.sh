#!/bin/bash
# GPU suite + smoke + bench of the in-tree build, then the A/B of build_variants/*.so against it
set -o pipefail
TAG=r7f bash scripts/gpu_check.sh || exit 1
TAG=r7f BS="65536 4096" ENVS=ant_heavenhell ENVS2="ant_tag" BS2="65536 8192" bash scripts/gpu_ab.sh
