# A/B: sixteen-lane kernel wall walk (unrolled register rows vs per-lane LDS walk), B = 4 096
set -o pipefail
mkdir -p gpurun_out/hexlw
for r in 1 2 3; do
  for env in ant_heavenhell ant_tag ant_gather; do
    for v in cur hexlw hexlw0; do
      env POB_LIB=$PWD/build_variants/$v.so timeout -k 10 120 python bench.py --no-cpu-baseline --steps 300 --env $env --global-batch 4096 \
        > gpurun_out/hexlw/$v.$env.4096.$r.json 2>/dev/null || exit 1
    done
  done
done
python - <<'PY'
import glob, json, collections, statistics
d = collections.defaultdict(list)
for f in glob.glob("gpurun_out/hexlw/*.json"):
    v, env, B, r = f.split("/")[-1][:-5].split(".")
    d[(env, int(B), v)].append(json.load(open(f))["roofline"]["kernel_ms"])
for k in sorted(d):
    print(*k, "median %.4f" % statistics.median(d[k]), sorted(d[k]))
PY
