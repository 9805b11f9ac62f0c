# Interleaved hex-vs-oct kernel choice over batch sizes (2 rounds, median kernel ms)
set -o pipefail
mkdir -p gpurun_out/selsw
for r in 1 2; do
  for env in ant_heavenhell ant_tag; do
    for B in 4096 5120 6144 7168; do
      for v in hex oct; do
        if [ $v = oct ]; then X="POB_HEXA_MAX_B=0"; else X="POB_HEXA_MAX_B=8192"; fi
        env $X timeout -k 10 120 python bench.py --no-cpu-baseline --steps 300 --env $env --batch $B \
          > gpurun_out/selsw/$v.$env.$B.$r.json 2>/dev/null || exit 1
      done
    done
  done
done
python - <<'PY'
import glob, json, collections, statistics
d = collections.defaultdict(list)
for f in glob.glob("gpurun_out/selsw/*.json"):
    v, env, B, r = f.split("/")[-1][:-5].split(".")
    j = json.load(open(f))
    d[(env, int(B), v)].append(j["roofline"]["kernel_ms"])
for k in sorted(d):
    print(*k, "median %.4f" % statistics.median(d[k]), sorted(d[k]))
PY
