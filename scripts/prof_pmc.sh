#!/bin/bash
# Kernel trace + PMC passes of one bench.py config into gpurun_out/prof_$TAG (each rocprofv3
# run under its own time limit; the chain stops at the first failure), then the summary
# profiles/$TAG_summary.md (profiles/summarize.py).
#   TAG=r3_hh4096 ARGS="--global-batch 4096" bash scripts/prof_pmc.sh
# SETS="A B C;D E" runs only those counter sets (';'-separated passes)
set -o pipefail
TAG=${TAG:?}
OUT=$PWD/gpurun_out/prof_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
B="python3 $PWD/bench.py --no-cpu-baseline --flop-envs 0 --steps 30 --warmup 3 $ARGS"
cd /tmp
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $OUT/trace -o trace --output-format csv -- $B > $OUT/trace.bench.json 2> $OUT/trace.err || { tail -5 $OUT/trace.err; exit 1; }
i=0
SETS_DEFAULT=1
[ -n "${SETS:-}" ] && SETS_DEFAULT=0
IFS=';' read -ra SETARR <<< "${SETS:-}"
[ $SETS_DEFAULT -eq 1 ] && SETARR=()
for set in "${SETARR[@]}"; do
  i=$((i + 1))
  timeout -s KILL 90 rocprofv3 --pmc $set -d $OUT/pmc$i -o pmc$i --output-format csv -- $B > $OUT/bench_pmc$i.json 2> $OUT/pmc$i.err || { tail -5 $OUT/pmc$i.err; exit 1; }
done
[ $SETS_DEFAULT -eq 1 ] && for set in "SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SALU" \
           "SQ_INSTS_SMEM SQ_INSTS_LDS SQ_INSTS_VMEM SQ_INSTS_BRANCH SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_SALU SQ_WAIT_INST_LDS" \
           "SQ_INSTS_VALU_TRANS_F32 SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_VMEM SQ_INST_CYCLES_SMEM SQ_IFETCH SQ_INSTS_VSKIPPED SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" \
           ${EXTRA_SETS:-FETCH_SIZE WRITE_SIZE}; do
  i=$((i + 1))
  timeout -s KILL 90 rocprofv3 --pmc $set -d $OUT/pmc$i -o pmc$i --output-format csv -- $B > $OUT/bench_pmc$i.json 2> $OUT/pmc$i.err || { tail -5 $OUT/pmc$i.err; exit 1; }
done
cd - > /dev/null
python3 profiles/summarize.py $OUT profiles/$TAG && cat profiles/${TAG}_summary.md | head -60
