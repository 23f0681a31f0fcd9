#!/bin/bash
# Build kernel variants of libmicrorts_amd.so into scripts/_exp/ for
# scripts/kernel_variants.py (A/B timing on the GPU box; not the product).
set -e
cd "$(dirname "$0")/.."
C=microrts-py_amd/csrc
F="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -mcode-object-version=5 -Iinclude -I$C -shared"
S="$C/mrts_engine.hip $C/mrts_bots.hip $C/mrts_capi.cpp"
build() { name=$1; shift; /opt/rocm/bin/hipcc $F "$@" -o scripts/_exp/lib_$name.so $S & }
build base

wait
ls -la scripts/_exp
