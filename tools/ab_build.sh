#!/bin/bash
# Build an A/B variant of libfdcn.so into build/ab/<name>/libfdcn.so with extra
# -D flags (e.g. tools/ab_build.sh nosplit -DFDCN_NO_SPLIT).  Time it on the
# GPU box with FDCN_LIB=build/ab/<name>/libfdcn.so python bench.py ...
set -e
NAME=$1; shift
cd "$(dirname "$0")/.."
mkdir -p build/ab/$NAME
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared "$@" \
  -o build/ab/$NAME/libfdcn.so finite_difference_amd/csrc/fdcn_kernels.hip \
  finite_difference_amd/csrc/fdcn_analytic.hip
