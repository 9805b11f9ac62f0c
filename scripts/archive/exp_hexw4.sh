#!/bin/bash
# A/B: the sixteen-lane kernel built for four waves per SIMD (POB_HEX_MINW=4, <= 128 VGPRs)
# at B = 16 384 (POB_HEXA_MAX_B=16384) against the default choice (eight-lane, two waves per SIMD)
set -o pipefail
mkdir -p gpurun_out/hexw4
for r in 1 2 3; do
  for env in ant_tag ant_heavenhell ant_gather; do
    timeout -k 10 120 python bench.py --no-cpu-baseline --steps 200 --env $env --global-batch 16384 > gpurun_out/hexw4/def.$env.$r.json 2>/dev/null || exit 1
    POB_LIB=$PWD/build_variants/hexw4.so POB_HEXA_MAX_B=16384 timeout -k 10 120 python bench.py --no-cpu-baseline --steps 200 --env $env --global-batch 16384 > gpurun_out/hexw4/w4.$env.$r.json 2>/dev/null || exit 1
  done
done
python - <<'PY'
import glob, json, collections, statistics
d = collections.defaultdict(list)
for f in glob.glob("gpurun_out/hexw4/*.json"):
    tag, env, r = f.split("/")[-1][:-5].split(".")
    j = json.load(open(f)); d[(env, tag)].append((j["roofline"]["kernel_ms"], j["roofline"]["kernel"]))
for k in sorted(d):
    print(*k, "median %.4f" % statistics.median(x[0] for x in d[k]), d[k][0][1])
PY
