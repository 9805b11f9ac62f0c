#!/bin/bash
# interleaved A/B of env-var settings: VARS="A=... ;B=..." (';'-separated), ENVS, BS, R
set -o pipefail
mkdir -p gpurun_out/abenv
IFS=';' read -ra VS <<< "$VARS"
for env in $ENVS; do for B in $BS; do for r in $(seq $R); do i=0; for v in "${VS[@]}"; do i=$((i+1))
  env $v timeout -k 10 120 python bench.py --no-cpu-baseline --flop-envs 0 --steps 200 --env $env --batch $B $EXTRA > gpurun_out/abenv/v$i.$env.$B.$r.json 2>/dev/null || exit 1
done; done; done; done
python3 - "$VARS" <<'PY'
import glob, json, collections, statistics, sys
names = sys.argv[1].split(';')
d = collections.defaultdict(list)
for f in glob.glob("gpurun_out/abenv/*.json"):
    v, env, B, r = f.split("/")[-1][:-5].split(".")
    d[(env, B, names[int(v[1:]) - 1])].append(json.load(open(f))["roofline"]["kernel_ms"])
for k in sorted(d): print(*k, "median %.4f" % statistics.median(d[k]), "runs", " ".join("%.4f" % x for x in sorted(d[k])))
PY
