set -o pipefail
mkdir -p gpurun_out
L=$PWD/build_variants/libpob_subt.so
POB_LIB=$L timeout -k 10 120 python scripts/sub_timing.py 4096 ant_heavenhell > gpurun_out/subt_hh4096.txt 2>&1 &&
POB_LIB=$L timeout -k 10 120 python scripts/sub_timing.py 8192 ant_tag > gpurun_out/subt_tag8192.txt 2>&1 &&
POB_LIB=$L timeout -k 10 120 python scripts/sub_timing.py 8192 ant_heavenhell > gpurun_out/subt_hh8192.txt 2>&1
cat gpurun_out/subt_*.txt
