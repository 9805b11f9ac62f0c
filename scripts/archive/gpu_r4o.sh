#!/bin/bash
# Round 4, final pass on the HEAD build: the GPU suite, smoke(), the candidate-skip A/B, the bench lines of every
# BASELINE config and of the per-GPU batches of the 1/2/4/8-GPU sweep, and PMC profiles of the
# eight- / sixteen-lane configs (the four-lane kernel is unchanged since profiles/r4m).
set -o pipefail
OUT=gpurun_out/r4o
mkdir -p $OUT
export TMPDIR=/tmp
python scripts/check_fresh.py || exit 3
fatal() { case $1 in 124|134|137|139) echo "fatal exit $1 in $2"; exit $1;; esac; }
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1; rc=$?; fatal $rc pytest
tail -2 $OUT/pytest_gpu.log; grep -E "FAILED|Error" $OUT/pytest_gpu.log | head -20
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1; rc=$?; fatal $rc smoke; tail -4 $OUT/smoke.log
# A/B: the exact candidate skips (libpob) against the build before them (build_variants/noskip.so)
rm -rf gpurun_out/ab
R=2 BS="65536 4096" ENVS="ant_heavenhell ant_tag" timeout -k 10 400 bash scripts/ab_bench.sh > $OUT/ab_skip.txt 2>&1; rc=$?; fatal $rc ab
cat $OUT/ab_skip.txt
for spec in "default:" "legacy:--legacy-spring" "hh_32768:--batch 32768" "hh_16384:--batch 16384" "hh_8192:--batch 8192" "hh_4096:--global-batch 4096" \
            "tag_65536:--env ant_tag" "tag_32768:--env ant_tag --batch 32768" "tag_16384:--env ant_tag --batch 16384" "tag_8192:--env ant_tag --global-batch 8192" \
            "ga_16384:--env ant_gather --global-batch 16384" "mixed_f16_32768:--env mixed --qp-dtype f16 --global-batch 32768" "gym_hh:--gym"; do
  name=${spec%%:*}; args=${spec#*:}
  cb="--no-cpu-baseline"; [ "$name" = "default" ] && cb=""; [ "$name" = "legacy" ] && cb=""
  timeout -k 10 300 python bench.py $cb $args > $OUT/bench_$name.json 2> $OUT/bench_$name.err || { tail -5 $OUT/bench_$name.err; exit 1; }
  python -c "import json; d=json.load(open('$OUT/bench_$name.json')); print('$name', '%.3e' % d['value'], d['roofline']['kernel_ms'])"
done
for spec in "r4o_hh4096:--global-batch 4096" "r4o_tag8192:--env ant_tag --global-batch 8192" "r4o_ga16384:--env ant_gather --global-batch 16384"; do
  tag=${spec%%:*}; args=${spec#*:}
  TAG=$tag ARGS="$args" timeout -k 10 600 bash scripts/prof_pmc.sh > $OUT/prof_$tag.log 2>&1 || { tail -20 $OUT/prof_$tag.log; exit 1; }
  echo "profiled $tag"
done
