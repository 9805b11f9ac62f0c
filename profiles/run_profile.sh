#!/bin/bash
# Profile one bench config on the GPU box (invoked through gpurun):
#   kernel-trace + stats (durations), then separate --pmc passes (HBM bytes, VALU work)
# as MI355X_MICROARCH.md §HBM / rocprofv3 prescribes.  Outputs land in gpurun_out/$TAG/.
# Usage: profiles/run_profile.sh TAG [bench.py args...]   (default: the headline config)
set -u
TAG=${1:-prof}
shift || true
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
ARGS="--steps 30 --warmup 3 --no-cpu-baseline $*"
run() {  # name, rocprofv3 args...
  local name=$1; shift
  timeout -k 10 300 rocprofv3 "$@" -d "$OUT/$name" -o "$name" --output-format csv -- \
      python3 "$ROOT/bench.py" $ARGS > "$OUT/$name.bench.json" 2> "$OUT/$name.err"
  local rc=$?
  echo "$name rc=$rc"
  return $rc
}
run trace --kernel-trace --stats &&
run pmc_fetch --pmc FETCH_SIZE &&
run pmc_write --pmc WRITE_SIZE &&
run pmc_valu --pmc SQ_INSTS_VALU SQ_WAVES SQ_INSTS_SALU SQ_INSTS_LDS GRBM_GUI_ACTIVE &&
run pmc_busy --pmc SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_VALU &&
run pmc_stall --pmc SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU_TRANS_F SQ_INSTS_SMEM SQ_INSTS_VMEM
