#!/bin/bash
# Round 4 measurement pass (mesh contacts, cooperative walk, stored contacts): bench lines of every BASELINE config,
# PMC profiles of the step kernels, and the FETCH_SIZE calibration microbenchmark.
set -o pipefail
OUT=gpurun_out/${TAG:-r4m}
mkdir -p $OUT
export TMPDIR=/tmp
python scripts/check_fresh.py || exit 3
for spec in "default:" "hh_4096:--global-batch 4096" "ga_16384:--env ant_gather --global-batch 16384" "tag_8192:--env ant_tag --global-batch 8192" "tag_65536:--env ant_tag" "mixed_f16_32768:--env mixed --qp-dtype f16 --global-batch 32768" "legacy:--legacy-spring" "gym_hh:--gym --no-cpu-baseline"; do
  name=${spec%%:*}; args=${spec#*:}
  cb="--no-cpu-baseline"; [ "$name" = "default" ] && cb=""; [ "$name" = "legacy" ] && cb=""
  timeout -k 10 300 python bench.py $cb $args > $OUT/bench_$name.json 2> $OUT/bench_$name.err || { tail -5 $OUT/bench_$name.err; exit 1; }
  python -c "import json; d=json.load(open('$OUT/bench_$name.json')); print('$name', '%.3e' % d['value'], d['roofline']['kernel_ms'])"
done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -o $OUT/fetch_cal scripts/fetch_calibration.hip || exit 1
cd /tmp
timeout -s KILL 60 rocprofv3 --pmc FETCH_SIZE -d $GRAFT_REPO_ROOT/$OUT/cal_fetch -o cal --output-format csv -- $GRAFT_REPO_ROOT/$OUT/fetch_cal > $GRAFT_REPO_ROOT/$OUT/cal.log 2>&1 || { tail -5 $GRAFT_REPO_ROOT/$OUT/cal.log; exit 1; }
timeout -s KILL 60 rocprofv3 --pmc WRITE_SIZE -d $GRAFT_REPO_ROOT/$OUT/cal_write -o cal --output-format csv -- $GRAFT_REPO_ROOT/$OUT/fetch_cal > $GRAFT_REPO_ROOT/$OUT/cal2.log 2>&1 || { tail -5 $GRAFT_REPO_ROOT/$OUT/cal2.log; exit 1; }
cd - > /dev/null
for spec in "r4m_hh65536:" "r4m_hh4096:--global-batch 4096" "r4m_tag8192:--env ant_tag --global-batch 8192" "r4m_ga16384:--env ant_gather --global-batch 16384" "r4m_legacy_hh65536:--legacy-spring"; do
  tag=${spec%%:*}; args=${spec#*:}
  TAG=$tag ARGS="$args" timeout -k 10 600 bash scripts/prof_pmc.sh > $OUT/prof_$tag.log 2>&1 || { tail -20 $OUT/prof_$tag.log; exit 1; }
  echo "profiled $tag"
done
