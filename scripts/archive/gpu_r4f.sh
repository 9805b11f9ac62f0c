#!/bin/bash
# Round 4: where the step time goes after the mesh contact port -- each config timed with the
# product build and timing-experiment builds (build_variants_t/: no wall contacts, no face walk
# (broadphase + face cull only), no velocity-pass re-walk, no physics), interleaved twice;
# then per-wave phase clocks (POB_EXP_TIMING build) for HH B = 4 096 and TAG B = 8 192.
OUT=gpurun_out/r4f
mkdir -p $OUT
export TMPDIR=/tmp
python scripts/check_fresh.py || exit 3
P=po-brax_amd/po_brax_amd/libpob.so; T=build_variants_t
run() {  # env B lib r
  local tag=$(basename $3 .so)
  POB_LIB=$PWD/$3 timeout -k 10 120 python bench.py --no-cpu-baseline --steps 200 --env $1 --batch $2 \
    > $OUT/$tag.$1.$2.$4.json 2> $OUT/$tag.$1.$2.$4.err || { tail -5 $OUT/$tag.$1.$2.$4.err; exit 1; }
}
for r in 1 2; do
  for cfg in "ant_heavenhell 4096" "ant_tag 8192" "ant_gather 16384"; do
    for lib in $P $T/nowalls.so $T/nophys.so; do run $cfg $lib $r; done
  done
  for cfg in "ant_heavenhell 65536" "ant_tag 65536"; do
    for lib in $P $T/nowalls.so $T/nowalk.so $T/novwalk.so $T/nophys.so; do run $cfg $lib $r; done
  done
  echo "round $r done"
done
python - <<'PY'
import glob, json, collections, statistics
d = collections.defaultdict(list)
for f in glob.glob("gpurun_out/r4f/*.json"):
    tag, env, B, r = f.split("/")[-1][:-5].rsplit(".", 3)
    d[(env, int(B), tag)].append(json.load(open(f))["roofline"]["kernel_ms"])
for k in sorted(d):
    print(k[0], k[1], k[2], "median kernel ms %.4f" % statistics.median(d[k]), ["%.4f" % x for x in d[k]])
PY
for cfg in "4096 ant_heavenhell" "8192 ant_tag"; do
  set -- $cfg
  POB_LIB=$PWD/$T/timing.so timeout -k 10 120 python scripts/phase_timing.py $1 $2 > $OUT/phase_$2_$1.txt 2>&1 || { tail -5 $OUT/phase_$2_$1.txt; exit 1; }
  echo "== phase $2 $1"; tail -12 $OUT/phase_$2_$1.txt
done
