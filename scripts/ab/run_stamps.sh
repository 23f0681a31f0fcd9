#!/bin/bash
# experiment: the stamp-instrumented build's phase breakdown of the fused k_step (configs[1])
set -euo pipefail
cd "${GRAFT_REPO_ROOT}"
O=gpurun_out/${1:-stamps}; mkdir -p $O
L=microrts-py_amd/gym_microrts/libmicrorts_amd.so
cp $L $O/../lib_product_backup.so 2>/dev/null || true
cp scripts/ab/${2:-libstamp.so} $L
timeout -k 10 300 python scripts/ab/stamps_runner.py 1024 coacAI > $O/stamps.txt 2>&1
cat $O/stamps.txt
