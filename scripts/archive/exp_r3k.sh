# round-3 kernel-selection change: the affected parity tests + bench lines
set -o pipefail
mkdir -p gpurun_out/r3k
timeout -k 10 900 python -u -m pytest tests/test_gpu_headline_parity.py -x -v --timeout 300 --timeout-method thread \
  -k "sixteen or eight or switch or wall_stress or config4" > gpurun_out/r3k/pytest_sel.log 2>&1 || { tail -30 gpurun_out/r3k/pytest_sel.log; exit 1; }
tail -3 gpurun_out/r3k/pytest_sel.log
for a in "ant_heavenhell 8192" "ant_tag 8192" "ant_gather 8192" "ant_heavenhell 4096"; do
  set -- $a
  timeout -k 10 120 python bench.py --no-cpu-baseline --steps 300 --env $1 --global-batch $2 > gpurun_out/r3k/bench_$1_$2.json || exit 1
  python -c "import json; d=json.load(open('gpurun_out/r3k/bench_$1_$2.json')); print('$1 $2', d['ms_per_step'], d['roofline']['kernel'], d['roofline']['kernel_ms'])"
done
