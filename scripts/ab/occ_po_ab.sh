#!/bin/bash
# EXPERIMENT: k_step at 8 workgroups / CU (launch_bounds(256, 8) + 78 SGPRs) vs the product,
# on configs[3]'s env part (partial obs, 4096 / 8192 envs), the headline and configs[1].
set -euo pipefail
cd "${GRAFT_REPO_ROOT}"
O=gpurun_out/$1; mkdir -p $O
L=microrts-py_amd/gym_microrts/libmicrorts_amd.so
cp $L /tmp/lib_product.so
cp scripts/ab/libw8.so $L
if ! timeout -k 10 400 python scripts/ab/quick_parity.py > $O/parity_w8.txt 2>&1; then echo "PARITY FAIL"; tail -5 $O/parity_w8.txt; cp /tmp/lib_product.so $L; exit 1; fi
timeout -k 10 400 python -m pytest tests/test_gpu_fullsize.py -m gpu -q -k "partial" > $O/parity_po_w8.txt 2>&1 || { echo "PO PARITY FAIL"; tail -5 $O/parity_po_w8.txt; cp /tmp/lib_product.so $L; exit 1; }
echo "parity ok: $(tail -1 $O/parity_po_w8.txt)"
for r in 1 2; do
  for v in base w8; do
    cp scripts/ab/lib$v.so $L
    for spec in "partial_obs 4096" "partial_obs 8192" "selfplay 8192" "coac 1024"; do
      set -- $spec
      timeout -k 10 300 python bench.py --workload $1 --envs-per-gpu $2 --steps 200 --warmup 30 --no-cpu-baseline > $O/${1}_$2_$v.$r.json 2>/dev/null
      python -c "import json; d=json.load(open('$O/${1}_$2_$v.$r.json')); print('$v r$r $1@$2', round(d['value']/1e6,2), round(d['kernels']['step']['avg_ms']*1000,1))"
    done
  done
done
cp /tmp/lib_product.so $L
