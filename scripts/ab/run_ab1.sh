#!/bin/bash
set -euo pipefail
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out/ab1
L=microrts-py_amd/gym_microrts/libmicrorts_amd.so
cp $L /tmp/lib_product.so
cp scripts/ab/libsetupwg.so $L
timeout -k 10 400 python scripts/ab/quick_parity.py > gpurun_out/ab1/parity_setupwg.txt 2>&1 || { tail -20 gpurun_out/ab1/parity_setupwg.txt; cp /tmp/lib_product.so $L; exit 1; }
tail -1 gpurun_out/ab1/parity_setupwg.txt
cp /tmp/lib_product.so $L
bash scripts/ab/ab.sh ab1 "base pb setupwg base_stamp setupwg_stamp" 2
