# eight-lane kernel at two waves per SIMD (B = 16 384): branch guards (default) vs GuardAcc forced
set -o pipefail
mkdir -p gpurun_out/octg
for r in 1 2 3; do
  for env in ant_gather ant_heavenhell ant_tag; do
    for v in br acc; do
      if [ $v = acc ]; then X="POB_OCT_GACC=1"; else X="POB_OCT_GACC=0"; fi
      env $X timeout -k 10 120 python bench.py --no-cpu-baseline --steps 300 --env $env --global-batch 16384 \
        > gpurun_out/octg/$v.$env.16384.$r.json 2>/dev/null || exit 1
    done
  done
done
python - <<'PY'
import glob, json, collections, statistics
d = collections.defaultdict(list)
for f in glob.glob("gpurun_out/octg/*.json"):
    v, env, B, r = f.split("/")[-1][:-5].split(".")
    d[(env, int(B), v)].append(json.load(open(f))["roofline"]["kernel_ms"])
for k in sorted(d):
    print(*k, "median %.4f" % statistics.median(d[k]), sorted(d[k]))
PY
