# A/B of the eight-lane kernel's HH build (per-lane LDS wall walk + register scalars)
set -o pipefail
mkdir -p gpurun_out/oct2
for r in 1 2 3; do
  for env in ant_heavenhell; do
    for B in 8192 16384; do
      for v in base oct2 oct2br; do
        case $v in base) X="POB_LIB=$PWD/build_variants/base.so";; oct2) X="POB_LIB=$PWD/build_variants/oct2.so";; oct2br) X="POB_LIB=$PWD/build_variants/oct2.so POB_OCT_GACC=0";; esac
        env $X timeout -k 10 120 python bench.py --no-cpu-baseline --steps 300 --env $env --global-batch $B \
          > gpurun_out/oct2/$v.$env.$B.$r.json 2>/dev/null || exit 1
      done
    done
  done
done
python - <<'PY'
import glob, json, collections, statistics
d = collections.defaultdict(list)
for f in glob.glob("gpurun_out/oct2/*.json"):
    v, env, B, r = f.split("/")[-1][:-5].split(".")
    d[(env, int(B), v)].append(json.load(open(f))["roofline"]["kernel_ms"])
for k in sorted(d):
    print(*k, "median %.4f" % statistics.median(d[k]), sorted(d[k]))
PY
