#!/bin/bash
# EXPERIMENT: segment order of the merged 8x8 + 16x16 launch (MRTS_EXP_ORDER), configs[4].
set -euo pipefail
cd "${GRAFT_REPO_ROOT}"
O=gpurun_out/$1; mkdir -p $O
L=microrts-py_amd/gym_microrts/libmicrorts_amd.so
cp $L /tmp/lib_product.so
cp scripts/ab/libord.so $L
for m in 1 2 3; do
  MRTS_EXP_ORDER=$m timeout -k 10 300 python -m pytest tests/test_gpu_bots.py -m gpu -q -k "mixed_map_buckets and False-5" > $O/parity_$m.txt 2>&1 && echo "parity ok $m" || { echo "PARITY FAIL $m"; tail -5 $O/parity_$m.txt; cp /tmp/lib_product.so $L; exit 1; }
done
for r in 1 2; do
  for m in 0 1 2 3; do
    MRTS_EXP_ORDER=$m timeout -k 10 300 python bench.py --workload mixed --no-cpu-baseline --steps 200 --warmup 30 > $O/mixed_$m.$r.json 2>/dev/null
    python -c "import json; d=json.load(open('$O/mixed_$m.$r.json')); print('order $m r$r', round(d['value']/1e6,2), d['roofline']['avg_launch_ms'])"
  done
done
cp /tmp/lib_product.so $L
