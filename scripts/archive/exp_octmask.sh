# eight-lane detection: per-slot wall masks (current) vs one mask over both centres' AABB (cur.so)
set -o pipefail
mkdir -p gpurun_out/octmask
timeout -k 10 600 python -u -m pytest tests/test_gpu_headline_parity.py -x -v --timeout 300 --timeout-method thread \
  -k "eight or wall_stress or out_of_range or free_running or octet or config4" > gpurun_out/octmask/pytest.log 2>&1 || { grep -E "^E |FAILED|Error" gpurun_out/octmask/pytest.log | head -30; exit 1; }
tail -1 gpurun_out/octmask/pytest.log
for r in 1 2 3; do
  for spec in "hh8192:--global-batch,8192" "tag8192:--env,ant_tag,--global-batch,8192" "ga8192:--env,ant_gather,--global-batch,8192" "hh16384:--global-batch,16384" "ga16384:--env,ant_gather,--global-batch,16384" "tag16384:--env,ant_tag,--global-batch,16384"; do
    name=${spec%%:*}; args=${spec#*:}; args=${args//,/ }
    for v in cur new; do
      if [ $v = cur ]; then X="POB_LIB=$PWD/build_variants/cur.so"; else X=""; fi
      env $X timeout -k 10 120 python bench.py --no-cpu-baseline --steps 300 $args > gpurun_out/octmask/$v.$name.$r.json 2>/dev/null || exit 1
    done
  done
done
python - <<'PY'
import glob, json, collections, statistics
d = collections.defaultdict(list)
for f in glob.glob("gpurun_out/octmask/*.json"):
    v, name, r = f.split("/")[-1][:-5].split(".")
    d[(name, v)].append(json.load(open(f))["roofline"]["kernel_ms"])
for k in sorted(d):
    print(*k, "median %.4f" % statistics.median(d[k]), sorted(d[k]))
PY
