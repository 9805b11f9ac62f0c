# four-lane kernel issue-priority schedules: cur (quartiles), prio2 (last three substeps), prio3 (last six, two each)
set -o pipefail
mkdir -p gpurun_out/prio2
for r in 1 2 3; do
  for spec in "hh65536:" "tag65536:--env,ant_tag" "mixed32768:--env,mixed,--qp-dtype,f16,--global-batch,32768" "ga65536:--env,ant_gather"; do
    name=${spec%%:*}; args=${spec#*:}; args=${args//,/ }
    for v in cur prio2 prio3; do
      POB_LIB=$PWD/build_variants/$v.so timeout -k 10 120 python bench.py --no-cpu-baseline --steps 300 $args > gpurun_out/prio2/$v.$name.$r.json 2>/dev/null || exit 1
    done
  done
done
python - <<'PY'
import glob, json, collections, statistics
d = collections.defaultdict(list)
for f in glob.glob("gpurun_out/prio2/*.json"):
    v, name, r = f.split("/")[-1][:-5].split(".")
    d[(name, v)].append(json.load(open(f))["roofline"]["kernel_ms"])
for k in sorted(d):
    print(*k, "median %.4f" % statistics.median(d[k]), sorted(d[k]))
PY
