#!/bin/bash
# Round 4: the four-lane velocity pass from the recorded winning candidates -- the GPU suite,
# A/B against the build before it (build_variants/skiponly.so), PMC profiles of the four-lane
# and legacy headline configs on this build, and their bench lines.
set -o pipefail
OUT=gpurun_out/r4q
mkdir -p $OUT
export TMPDIR=/tmp
python scripts/check_fresh.py || exit 3
fatal() { case $1 in 124|134|137|139) echo "fatal exit $1 in $2"; exit $1;; esac; }
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1; rc=$?; fatal $rc pytest
tail -2 $OUT/pytest_gpu.log; grep -E "FAILED|Error" $OUT/pytest_gpu.log | head -20
[ $rc -ne 0 ] && exit $rc
rm -rf gpurun_out/ab
R=3 BS="65536" ENVS="ant_heavenhell ant_tag" timeout -k 10 400 bash scripts/ab_bench.sh > $OUT/ab_kinds.txt 2>&1; rc=$?; fatal $rc ab
cat $OUT/ab_kinds.txt
for spec in "r4q_hh65536:" "r4q_legacy_hh65536:--legacy-spring"; do
  tag=${spec%%:*}; args=${spec#*:}
  TAG=$tag ARGS="$args" timeout -k 10 600 bash scripts/prof_pmc.sh > $OUT/prof_$tag.log 2>&1 || { tail -20 $OUT/prof_$tag.log; exit 1; }
  echo "profiled $tag"
done
