set -o pipefail
mkdir -p gpurun_out/dbg
timeout -k 10 300 python scripts/debug_mismatch.py ant_heavenhell 65536 > gpurun_out/dbg/log.txt 2>&1; cat gpurun_out/dbg/log.txt | tail -5
