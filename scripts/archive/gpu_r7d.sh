set -o pipefail
mkdir -p gpurun_out/r7d
timeout -k 10 420 python -u scripts/episode_bench.py > gpurun_out/r7d/episode_hh65536.json 2> gpurun_out/r7d/episode.err || { tail -20 gpurun_out/r7d/episode.err; exit 1; }
R=3 BS="65536 4096" ENVS="ant_heavenhell" STEPS=100 bash scripts/ab_bench.sh > gpurun_out/r7d/ab.txt 2>&1 || { tail gpurun_out/r7d/ab.txt; exit 1; }
cat gpurun_out/r7d/ab.txt
for env in ant_heavenhell ant_tag; do for B in 65536 32768 16384 8192; do
  timeout -k 10 120 python bench.py --no-cpu-baseline --flop-envs 0 --steps 200 --env $env --global-batch $B > gpurun_out/r7d/sweep_${env}_$B.json 2>/dev/null || exit 1
  python -c "import json,sys; j=json.load(open('gpurun_out/r7d/sweep_${env}_$B.json')); print('$env', $B, j['roofline']['kernel_ms'], j['value'])"
done; done
