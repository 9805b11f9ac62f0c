#!/bin/bash
# Round 4: instruction-cache counters of the HH 65536 quad kernel (is SQ_WAIT_INST_ANY, 27 % of
# wave-cycles in profiles/r4p_hh65536_summary.md, instruction-fetch misses?), one PMC pass each.
set -o pipefail
OUT=gpurun_out/r4t
mkdir -p $OUT
export TMPDIR=/tmp
python scripts/check_fresh.py || exit 3
TAG=r4t_hh65536 ARGS="" SETS="SQC_ICACHE_REQ SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE;SQC_DCACHE_REQ SQC_DCACHE_HITS SQC_DCACHE_MISSES SQ_WAIT_INST_ANY" \
  timeout -k 10 400 bash scripts/prof_pmc.sh > $OUT/prof.log 2>&1; rc=$?
tail -40 $OUT/prof.log
exit $rc
