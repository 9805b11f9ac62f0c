# eight-lane kernel at two waves per SIMD: falling issue priority (new, committed form) vs none (cur): parity subset + kernel ms
set -o pipefail
mkdir -p gpurun_out/octprio2
timeout -k 10 600 python -u -m pytest tests/test_gpu_headline_parity.py -x -v --timeout 300 --timeout-method thread -k "eight or octet or wall_stress or out_of_range or free_running or bench_sizes or config4" > gpurun_out/octprio2/pytest.log 2>&1 || { grep -E "^E |FAILED|Error" gpurun_out/octprio2/pytest.log | head -30; exit 1; }
tail -1 gpurun_out/octprio2/pytest.log
for r in 1 2 3; do
  for spec in "hh16384:--global-batch,16384" "ga16384:--env,ant_gather,--global-batch,16384" "tag16384:--env,ant_tag,--global-batch,16384" "hh12288:--global-batch,12288" "tag8192:--env,ant_tag,--global-batch,8192"; do
    name=${spec%%:*}; args=${spec#*:}; args=${args//,/ }
    for v in cur new; do
      if [ $v = cur ]; then X="POB_LIB=$PWD/build_variants/cur.so"; else X=""; fi
      env $X timeout -k 10 120 python bench.py --no-cpu-baseline --steps 300 $args > gpurun_out/octprio2/$v.$name.$r.json 2>/dev/null || exit 1
    done
  done
done
python - <<'PY'
import glob, json, collections, statistics
d = collections.defaultdict(list)
for f in glob.glob("gpurun_out/octprio2/*.json"):
    v, name, r = f.split("/")[-1][:-5].split(".")
    d[(name, v)].append(json.load(open(f))["roofline"]["kernel_ms"])
for k in sorted(d):
    print(*k, "median %.4f" % statistics.median(d[k]), sorted(d[k]))
PY
