#!/bin/bash
# GPU suite + smoke + bench, then the PMC profiles of three BASELINE configs
set -o pipefail
TAG=r7l bash scripts/gpu_check.sh || exit 1
R=r7l bash scripts/gpu_prof_all.sh hh65536 hh4096_mask ga16384
