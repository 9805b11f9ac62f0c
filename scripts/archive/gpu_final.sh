# Round-end GPU record: full -m gpu suite, smoke(), one bench line per BASELINE config (and the
# gym path), all into gpurun_out/$TAG/.  Every GPU step has its own time limit; the chain
# stops at the first failure.
set -o pipefail
TAG=${TAG:-r3_final}
K="not zzz_none" TAG=$TAG BENCHES="default: hh_4096:--global-batch,4096 ga_16384:--env,ant_gather,--global-batch,16384 tag_65536:--env,ant_tag tag_8192:--env,ant_tag,--global-batch,8192 mixed_f16_32768:--env,mixed,--qp-dtype,f16,--global-batch,32768 gym_hh_65536:--gym gym_ga_16384:--gym,--env,ant_gather,--global-batch,16384 gym_tag_65536:--gym,--env,ant_tag" bash scripts/gpu_r3.sh || exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/$TAG/smoke.log 2>&1 || { tail -20 gpurun_out/$TAG/smoke.log; exit 1; }
tail -4 gpurun_out/$TAG/smoke.log
timeout -k 10 300 python bench.py > gpurun_out/$TAG/bench_default_with_cpu.json 2> gpurun_out/$TAG/bench_default_with_cpu.err || { tail -5 gpurun_out/$TAG/bench_default_with_cpu.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/$TAG/bench_default_with_cpu.json')); print('default+cpu', d['value'], d['cpu_baseline']['value'] if d['cpu_baseline'] else None)"
