# hipGraph replay vs eager back-to-back launches (wall-clock ms per step), interleaved, 3 rounds
set -o pipefail
mkdir -p gpurun_out/gve
for r in 1 2 3; do
  for spec in "hh65536:" "tag65536:--env,ant_tag" "hh4096:--global-batch,4096" "ga16384:--env,ant_gather,--global-batch,16384" "hh16384:--global-batch,16384"; do
    name=${spec%%:*}; args=${spec#*:}; args=${args//,/ }
    for v in graph eager; do
      if [ $v = eager ]; then X="--no-graph"; else X=""; fi
      timeout -k 10 120 python bench.py --no-cpu-baseline --steps 500 $args $X > gpurun_out/gve/$v.$name.$r.json 2>/dev/null || exit 1
    done
  done
done
python - <<'PY'
import glob, json, collections, statistics
d = collections.defaultdict(list)
for f in glob.glob("gpurun_out/gve/*.json"):
    v, name, r = f.split("/")[-1][:-5].split(".")
    j = json.load(open(f))
    d[(name, v)].append((j["ms_per_step"], j["roofline"]["kernel_ms"], j["roofline"].get("eager_event_ms")))
for k in sorted(d):
    print(*k, "wall median %.4f" % statistics.median(x[0] for x in d[k]), "kernel %.4f" % statistics.median(x[1] for x in d[k]), "eager_ev %.4f" % statistics.median(x[2] for x in d[k]))
PY
