#!/bin/bash
# Round 4: the small-batch floor decomposition -- configs 2 / 3 / 4's per-GPU batch timed with
# the product build, a build without wall contacts and one without physics
# (build_variants_t/, timing experiments), interleaved three times; then per-wave phase clocks
# (POB_EXP_TIMING build) for HH B = 4 096 and TAG B = 8 192.
OUT=gpurun_out/r4f
mkdir -p $OUT
export TMPDIR=/tmp
python scripts/check_fresh.py || exit 3
for r in 1 2 3; do
  for cfg in "ant_heavenhell 4096" "ant_tag 8192" "ant_gather 16384"; do
    set -- $cfg
    for lib in po-brax_amd/po_brax_amd/libpob.so build_variants_t/nowalls.so build_variants_t/nophys.so; do
      tag=$(basename $lib .so)
      POB_LIB=$PWD/$lib timeout -k 10 120 python bench.py --no-cpu-baseline --steps 300 --env $1 --batch $2 \
        > $OUT/$tag.$1.$2.$r.json 2> $OUT/$tag.$1.$2.$r.err || { tail -5 $OUT/$tag.$1.$2.$r.err; exit 1; }
    done
  done
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
  POB_LIB=$PWD/build_variants_t/timing.so timeout -k 10 120 python scripts/phase_timing.py $1 $2 > $OUT/phase_$2_$1.txt 2>&1 || { tail -5 $OUT/phase_$2_$1.txt; exit 1; }
  echo "== phase $2 $1"; tail -12 $OUT/phase_$2_$1.txt
done
