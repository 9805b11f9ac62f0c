#!/bin/bash
# Interleaved A/B timing of libpob.so builds (default + build_variants/*.so), R rounds each,
# one bench.py process per (round, lib); prints the per-lib median kernel ms.
#   R=3 BS="65536" ENVS="ant_heavenhell" bash scripts/ab_bench.sh
set -o pipefail
shopt -s nullglob
mkdir -p gpurun_out/ab
R=${R:-3}
# (a directory build_variants/NAME/ holding a whole po_brax_amd package with its libpob.so is
# run as variant NAME through POB_PKG_ROOT: A/B of Python-side changes too)
libs="po-brax_amd/po_brax_amd/libpob.so $(echo build_variants/*.so build_variants/*/)"  # (nullglob)
for env in ${ENVS:-ant_heavenhell}; do
  for B in ${BS:-65536}; do
    for r in $(seq $R); do
      for lib in $libs; do
        tag=$(basename $lib .so)
        if [ -d $lib ]; then pk="POB_PKG_ROOT=$PWD/$lib POB_LIB=$PWD/$lib/po_brax_amd/libpob.so"; else pk="POB_LIB=$PWD/$lib"; fi
        env $pk timeout -k 10 120 python bench.py --no-cpu-baseline --flop-envs 0 --steps ${STEPS:-200} --env $env --batch $B ${EXTRA:-} \
          > gpurun_out/ab/$tag.$env.$B.$r.json 2>/dev/null || exit 1
      done
    done
  done
done
python - <<'PY'
import glob, json, collections, os, statistics
d = collections.defaultdict(list)
for f in glob.glob("gpurun_out/ab/*.json"):
    tag, env, B, r = f.split("/")[-1][:-5].rsplit(".", 3)
    j = json.load(open(f))
    d[(env, B, tag)].append(j["ms_per_step"] if os.environ.get("FIELD") == "step" else j["roofline"]["kernel_ms"])
for k in sorted(d):
    print(*k, "median %.4f" % statistics.median(d[k]), "runs", " ".join("%.4f" % x for x in sorted(d[k])))
PY
