#!/bin/bash
set -euo pipefail
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out/ab2
L=microrts-py_amd/gym_microrts/libmicrorts_amd.so
cp $L /tmp/lib_product.so
cp scripts/ab/libbase_headstamp.so $L
timeout -k 10 300 python scripts/ab/stamps_head.py > gpurun_out/ab2/headstamps_base.json 2> gpurun_out/ab2/headstamps_base.err || true
cp /tmp/lib_product.so $L
bash scripts/ab/run_ab.sh ab2 "tr tr_nt64 att" "base tr tr_nt64 att tr_stamp" 2
