# eight-lane kernel at two waves per SIMD: falling issue priority (octprio) vs none (cur), kernel ms
set -o pipefail
mkdir -p gpurun_out/octprio
for r in 1 2 3; do
  for spec in "hh16384:--global-batch,16384" "ga16384:--env,ant_gather,--global-batch,16384" "tag16384:--env,ant_tag,--global-batch,16384" "hh12288:--global-batch,12288" "tag8192:--env,ant_tag,--global-batch,8192"; do
    name=${spec%%:*}; args=${spec#*:}; args=${args//,/ }
    for v in cur octprio; do
      POB_LIB=$PWD/build_variants/$v.so timeout -k 10 120 python bench.py --no-cpu-baseline --steps 300 $args > gpurun_out/octprio/$v.$name.$r.json 2>/dev/null || exit 1
    done
  done
done
python - <<'PY'
import glob, json, collections, statistics
d = collections.defaultdict(list)
for f in glob.glob("gpurun_out/octprio/*.json"):
    v, name, r = f.split("/")[-1][:-5].split(".")
    d[(name, v)].append(json.load(open(f))["roofline"]["kernel_ms"])
for k in sorted(d):
    print(*k, "median %.4f" % statistics.median(d[k]), sorted(d[k]))
PY
