# eight-lane kernel: register walls + GuardAcc + task prefetch -- parity subset, then A/B
set -o pipefail
mkdir -p gpurun_out/oct
timeout -k 10 900 python -u -m pytest tests/test_gpu_headline_parity.py -x -v --timeout 300 --timeout-method thread \
  -k "eight or octet or wall_stress or out_of_range or config4 or switch or bench_sizes" > gpurun_out/oct/pytest.log 2>&1 || { tail -30 gpurun_out/oct/pytest.log; exit 1; }
tail -2 gpurun_out/oct/pytest.log
for r in 1 2 3; do
  for env in ant_heavenhell ant_tag ant_gather; do
    for B in 8192 16384; do
      for v in base new newbr; do
        case $v in base) X="POB_LIB=$PWD/build_variants/base.so";; new) X="";; newbr) X="POB_OCT_GACC=0";; esac
        env $X timeout -k 10 120 python bench.py --no-cpu-baseline --steps 300 --env $env --global-batch $B \
          > gpurun_out/oct/$v.$env.$B.$r.json 2>/dev/null || exit 1
      done
    done
  done
done
python - <<'PY'
import glob, json, collections, statistics
d = collections.defaultdict(list)
for f in glob.glob("gpurun_out/oct/*.json"):
    v, env, B, r = f.split("/")[-1][:-5].split(".")
    d[(env, int(B), v)].append(json.load(open(f))["roofline"]["kernel_ms"])
for k in sorted(d):
    print(*k, "median %.4f" % statistics.median(d[k]), sorted(d[k]))
PY
