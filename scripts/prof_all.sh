#!/bin/bash
# PMC profiles of the BASELINE configs for the current build (scripts/prof_pmc.sh each; the
# chain stops at the first failure): profiles/${P}_<config>_summary.md / _traffic.json
#   P=r6n bash scripts/prof_all.sh
set -o pipefail
P=${P:?}
TAG=${P}_hh65536 ARGS="" bash scripts/prof_pmc.sh > /dev/null || exit 1
TAG=${P}_hh4096_mask ARGS="--env ant_heavenhell --global-batch 4096 --obs-mask no-cfrc" bash scripts/prof_pmc.sh > /dev/null || exit 1
TAG=${P}_tag8192 ARGS="--env ant_tag --global-batch 8192" bash scripts/prof_pmc.sh > /dev/null || exit 1
TAG=${P}_ga16384 ARGS="--env ant_gather --global-batch 16384" bash scripts/prof_pmc.sh > /dev/null || exit 1
TAG=${P}_tag65536 ARGS="--env ant_tag" bash scripts/prof_pmc.sh > /dev/null || exit 1
TAG=${P}_mixed32768 ARGS="--env mixed --qp-dtype f16 --global-batch 32768" bash scripts/prof_pmc.sh > /dev/null || exit 1
echo done
