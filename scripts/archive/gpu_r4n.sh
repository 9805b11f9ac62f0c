#!/bin/bash
# Round 4: A/B of the eight- / sixteen-lane kernels' per-body broadphase (libpob) against the
# build before it (build_variants/nobbox.so), and the bench lines after the round-4 profiles
# were committed (their traffic / VALU fields read them).
OUT=gpurun_out/r4n
mkdir -p $OUT
export TMPDIR=/tmp
python scripts/check_fresh.py || exit 3
fatal() { case $1 in 124|134|137|139) echo "fatal exit $1 in $2"; exit $1;; esac; }
rm -rf gpurun_out/ab
R=3 BS="4096 8192 16384" ENVS="ant_heavenhell ant_tag ant_gather" timeout -k 10 700 bash scripts/ab_bench.sh > $OUT/ab_bbox.txt 2>&1; rc=$?; fatal $rc ab
cat $OUT/ab_bbox.txt
timeout -k 10 300 python bench.py > $OUT/bench_default.json 2> $OUT/bench_default.err || { tail -5 $OUT/bench_default.err; exit 1; }
python -c "import json; d=json.load(open('$OUT/bench_default.json')); print(d['value'], d['roofline'])"
