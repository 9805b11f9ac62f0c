# Interleaved hex-vs-oct kernel choice at B = 8 192 (3 rounds, median kernel ms per env)
set -o pipefail
mkdir -p gpurun_out/sel
for r in 1 2 3; do
  for env in ant_heavenhell ant_tag ant_gather; do
    for v in hex oct; do
      if [ $v = oct ]; then X="POB_HEXA_MAX_B=0"; else X=""; fi
      env $X timeout -k 10 120 python bench.py --no-cpu-baseline --steps 300 --env $env --batch 8192 \
        > gpurun_out/sel/$v.$env.$r.json 2>/dev/null || exit 1
    done
  done
done
python - <<'PY'
import glob, json, collections, statistics
d = collections.defaultdict(list)
for f in glob.glob("gpurun_out/sel/*.json"):
    v, env, r = f.split("/")[-1][:-5].split(".")
    j = json.load(open(f))
    d[(env, v)].append((j["roofline"]["kernel_ms"], j["roofline"]["kernel"]))
for k in sorted(d):
    print(*k, "median %.4f" % statistics.median(x for x, _ in d[k]), sorted(x for x, _ in d[k]), d[k][0][1])
PY
