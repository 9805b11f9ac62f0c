set -o pipefail
mkdir -p gpurun_out
bash scripts/variant_bench_env.sh ant_heavenhell 65536 ant_heavenhell 4096 > gpurun_out/exp1_variants.txt 2>&1 || exit 1
POB_LIB=$PWD/build_variants/libpob_timing.so timeout -k 10 120 python scripts/phase_timing.py 65536 > gpurun_out/exp1_ts65536.txt 2>&1 || exit 1
POB_LIB=$PWD/build_variants/libpob_timing.so timeout -k 10 120 python scripts/phase_timing.py 4096 > gpurun_out/exp1_ts4096.txt 2>&1 || exit 1
cat gpurun_out/exp1_variants.txt gpurun_out/exp1_ts65536.txt gpurun_out/exp1_ts4096.txt
