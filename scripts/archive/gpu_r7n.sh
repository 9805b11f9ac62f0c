#!/bin/bash
# the rest of the PMC profiles, the batch sweep behind DESIGN §6's projection and a whole
# episode (scripts/episode_bench.py) on the in-tree build
set -o pipefail
R=r7l bash scripts/gpu_prof_all.sh tag65536 tag8192 mixed32768 || exit 1
mkdir -p gpurun_out/r7n
for env in ant_heavenhell ant_tag; do for B in 65536 32768 16384 8192; do
  timeout -k 10 120 python bench.py --no-cpu-baseline --flop-envs 0 --steps 200 --env $env --global-batch $B > gpurun_out/r7n/sweep_${env}_$B.json 2>/dev/null || exit 1
  python -c "import json; j=json.load(open('gpurun_out/r7n/sweep_${env}_$B.json')); print('$env', $B, j['roofline']['kernel_ms'], j['value'])"
done; done
timeout -k 10 420 python -u scripts/episode_bench.py > gpurun_out/r7n/episode_hh65536.json 2> gpurun_out/r7n/episode.err || { tail -20 gpurun_out/r7n/episode.err; exit 1; }
python -c "import json; j=json.load(open('gpurun_out/r7n/episode_hh65536.json')); print(j['ms_per_step_episode'], [w['ms_per_step'] for w in j['windows']])"
