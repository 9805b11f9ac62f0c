#!/bin/bash
# Round 4: PMC profiles of the four-lane and legacy headline configs on the final build
# (the candidate skips changed the four-lane kernel after profiles/r4m), then their bench lines
# (which read the newest committed profile of their config: rerun after committing).
set -o pipefail
OUT=gpurun_out/r4p
mkdir -p $OUT
export TMPDIR=/tmp
python scripts/check_fresh.py || exit 3
for spec in "r4p_hh65536:" "r4p_legacy_hh65536:--legacy-spring" "r4p_tag65536:--env ant_tag"; do
  tag=${spec%%:*}; args=${spec#*:}
  TAG=$tag ARGS="$args" timeout -k 10 600 bash scripts/prof_pmc.sh > $OUT/prof_$tag.log 2>&1 || { tail -20 $OUT/prof_$tag.log; exit 1; }
  echo "profiled $tag"
done
