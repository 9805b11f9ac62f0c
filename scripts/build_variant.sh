#!/bin/bash
# Build one experiment variant of libpob.so into build_variants/NAME.so:
#   bash scripts/build_variant.sh NAME -DPOB_EXP_...
set -e
NAME=$1; shift
cd "$(dirname "$0")/.."
mkdir -p build_variants
CS=po-brax_amd/csrc
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -fno-fast-math -fno-slp-vectorize \
  -fPIC -shared -mcode-object-version=5 -Wall -Wno-unused-result "$@" \
  -o build_variants/.$NAME.tmp $CS/pob_kernels.hip $CS/pob_system.cpp
mv build_variants/.$NAME.tmp build_variants/$NAME.so  # (atomic: a GPU snapshot never sees half a library)
