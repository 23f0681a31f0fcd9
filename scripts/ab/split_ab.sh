#!/bin/bash
# EXPERIMENT: the headline's last K games on two workgroups each (redundant logic, each
# streams half the outputs).  Quick parity at K=512 (the halves' race is not closed in
# this build: a mismatch there is the race, not the split), then interleaved benches.
set -euo pipefail
cd "${GRAFT_REPO_ROOT}"
O=gpurun_out/$1; mkdir -p $O
L=microrts-py_amd/gym_microrts/libmicrorts_amd.so
cp $L /tmp/lib_product.so
cp scripts/ab/libsplit.so $L
MRTS_EXP_SPLIT=512 timeout -k 10 300 python -m pytest tests/test_gpu_fullsize.py -m gpu -q -k "selfplay_8192" > $O/parity.txt 2>&1 && echo "parity ok" || { echo "parity FAIL"; tail -5 $O/parity.txt; }
for round in 1 2; do
  for K in 0 256 512 1024 1536; do
    MRTS_EXP_SPLIT=$K timeout -k 10 200 python bench.py --no-cpu-baseline --steps 200 > $O/head_$K.$round.json 2>/dev/null
    python -c "import json; d=json.load(open('$O/head_$K.$round.json')); print('K=$K r$round', round(d['value']/1e6,2), round(d['kernels']['step']['avg_ms']*1000,1))"
  done
done
cp /tmp/lib_product.so $L
