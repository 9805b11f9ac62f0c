# four-lane kernel: prologue at priority 3 (pstart) vs the default 0 (cur), kernel ms
set -o pipefail
mkdir -p gpurun_out/pstart
for r in 1 2 3; do
  for spec in "hh65536:" "tag65536:--env,ant_tag" "mixed32768:--env,mixed,--qp-dtype,f16,--global-batch,32768" "hh32768:--global-batch,32768"; do
    name=${spec%%:*}; args=${spec#*:}; args=${args//,/ }
    for v in cur pstart; do
      POB_LIB=$PWD/build_variants/$v.so timeout -k 10 120 python bench.py --no-cpu-baseline --steps 300 $args > gpurun_out/pstart/$v.$name.$r.json 2>/dev/null || exit 1
    done
  done
done
python - <<'PY'
import glob, json, collections, statistics
d = collections.defaultdict(list)
for f in glob.glob("gpurun_out/pstart/*.json"):
    v, name, r = f.split("/")[-1][:-5].split(".")
    d[(name, v)].append(json.load(open(f))["roofline"]["kernel_ms"])
for k in sorted(d):
    print(*k, "median %.4f" % statistics.median(d[k]), sorted(d[k]))
PY
