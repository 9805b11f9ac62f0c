# masked reset, AntGather: objects / object rows / readings one lane per object (current) vs the quad's loops (fill.so)
set -o pipefail
mkdir -p gpurun_out/gaobj
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread \
  -k "gym or autoreset or reset or randomized or eval or sharded or rollout or fp16 or mixed" > gpurun_out/gaobj/pytest.log 2>&1 || { grep -E "^E |FAILED|Error" gpurun_out/gaobj/pytest.log | head -30; exit 1; }
tail -1 gpurun_out/gaobj/pytest.log
for r in 1 2 3; do
  for spec in ant_gather:16384 ant_gather:65536; do
    env=${spec%%:*}; B=${spec#*:}
    for v in fill obj; do
      case $v in fill) X="POB_LIB=$PWD/build_variants/$v.so";; obj) X="";; esac
      env $X timeout -k 10 120 python bench.py --no-cpu-baseline --gym --steps 300 --env $env --global-batch $B \
        > gpurun_out/gaobj/$v.$env.$B.$r.json 2>/dev/null || exit 1
    done
  done
done
python - <<'PY'
import glob, json, collections, statistics
d = collections.defaultdict(list)
for f in glob.glob("gpurun_out/gaobj/*.json"):
    v, env, B, r = f.split("/")[-1][:-5].split(".")
    d[(env, int(B), v)].append(json.load(open(f))["ms_per_step"])
for k in sorted(d):
    print(*k, "median %.4f" % statistics.median(d[k]), sorted(d[k]))
PY
