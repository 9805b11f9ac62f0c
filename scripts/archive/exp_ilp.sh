# compiler scheduling strategy A/B: default (cur) vs -mllvm -amdgpu-sched-strategy=max-ilp (ilp), kernel ms
set -o pipefail
mkdir -p gpurun_out/ilp
for r in 1 2 3; do
  for spec in "hh65536:" "hh4096:--global-batch,4096" "tag8192:--env,ant_tag,--global-batch,8192" "ga16384:--env,ant_gather,--global-batch,16384" "hh32768:--global-batch,32768" "tag4096:--env,ant_tag,--global-batch,4096"; do
    name=${spec%%:*}; args=${spec#*:}; args=${args//,/ }
    for v in cur ilp; do
      POB_LIB=$PWD/build_variants/$v.so timeout -k 10 120 python bench.py --no-cpu-baseline --steps 300 $args > gpurun_out/ilp/$v.$name.$r.json 2>/dev/null || exit 1
    done
  done
done
python - <<'PY'
import glob, json, collections, statistics
d = collections.defaultdict(list)
for f in glob.glob("gpurun_out/ilp/*.json"):
    v, name, r = f.split("/")[-1][:-5].split(".")
    d[(name, v)].append(json.load(open(f))["roofline"]["kernel_ms"])
for k in sorted(d):
    print(*k, "median %.4f" % statistics.median(d[k]), sorted(d[k]))
PY
