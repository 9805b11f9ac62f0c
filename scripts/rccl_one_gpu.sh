#!/bin/bash
# RCCL on the one-GPU box: the sharded product path and the overlapped obs gather
# (scripts/multirank_check.py) over the nccl backend with one rank -- RCCL refuses two ranks on
# one device ("Duplicate GPU detected", profiles/r7v) -- and two ranks over gloo.  Stops at the
# first failure.
set -u
OUT=gpurun_out/${TAG:-rccl}
mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0
run() {  # name, seconds, command...
  local n=$1 s=$2; shift 2
  timeout -k 10 $s "$@" > $OUT/$n.txt 2>&1
  local rc=$?
  echo "$n rc=$rc"; grep "^multirank" $OUT/$n.txt
  return $rc
}
TR="python -m torch.distributed.run --nnodes=1 --master-addr 127.0.0.1"
run nccl_world1_hh 240 $TR --nproc-per-node 1 --master-port 29511 scripts/multirank_check.py --backend nccl --env ant_heavenhell || exit $?
run nccl_world1_tag 240 $TR --nproc-per-node 1 --master-port 29512 scripts/multirank_check.py --backend nccl --env ant_tag || exit $?
run gloo_world2_hh 240 $TR --nproc-per-node 2 --master-port 29513 scripts/multirank_check.py --backend gloo --env ant_heavenhell || exit $?
