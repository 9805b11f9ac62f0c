#!/bin/bash
# Kernel trace + PMC passes (scripts/prof_pmc.sh) of the BASELINE configs on the in-tree build,
# summaries into profiles/${R}_<config>_summary.md (R: the round-tag prefix, e.g. r7x); the
# configs to run as arguments (default: all six)
set -o pipefail
R=${R:?}
CFGS=${*:-"hh65536 hh4096_mask ga16384 tag65536 tag8192 mixed32768"}
for c in $CFGS; do
  case $c in
    hh65536) A="" ;;
    hh4096_mask) A="--global-batch 4096 --obs-mask no-cfrc" ;;
    ga16384) A="--env ant_gather --global-batch 16384" ;;
    tag65536) A="--env ant_tag" ;;
    tag8192) A="--env ant_tag --global-batch 8192" ;;
    mixed32768) A="--env mixed --qp-dtype f16 --global-batch 32768" ;;
    *) echo "unknown config $c"; exit 1 ;;
  esac
  TAG=${R}_$c ARGS="$A" bash scripts/prof_pmc.sh > gpurun_out/prof_${R}_$c.log 2>&1 || { tail -20 gpurun_out/prof_${R}_$c.log; exit 1; }
  grep -E "k_step|HBM bytes" profiles/${R}_${c}_summary.md | head -4
done
