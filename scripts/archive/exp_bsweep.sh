# throughput vs batch size (one box, one run each), HH / TAG / GA, default kernel selection
set -o pipefail
mkdir -p gpurun_out/bsweep
for env in ant_heavenhell ant_tag ant_gather; do
  for B in 256 1024 2048 4096 6144 8192 12288 16384 24576 32768 49152 65536 131072 262144; do
    timeout -k 10 150 python bench.py --no-cpu-baseline --steps 200 --env $env --global-batch $B > gpurun_out/bsweep/$env.$B.json 2>/dev/null || { echo fail $env $B; exit 1; }
  done
  echo done $env
done
python - <<'PY'
import glob, json
rows = []
for f in glob.glob("gpurun_out/bsweep/*.json"):
    env, B = f.split("/")[-1][:-5].split(".")
    j = json.load(open(f))
    rows.append((env, int(B), j["value"], j["ms_per_step"], j["roofline"]["kernel"], j["roofline"]["frac"]))
for r in sorted(rows):
    print("%-16s %7d %10.3e env-steps/s %8.4f ms %-28s frac %.3f" % r)
PY
