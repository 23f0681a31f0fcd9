#!/bin/bash
# run_ab.sh TAG "libs to parity-check" "libs to A/B" [rounds]
set -euo pipefail
cd "${GRAFT_REPO_ROOT}"
O=gpurun_out/$1; mkdir -p $O
L=microrts-py_amd/gym_microrts/libmicrorts_amd.so
cp $L /tmp/lib_product.so
for v in $2; do
  cp scripts/ab/lib$v.so $L
  if ! timeout -k 10 400 python scripts/ab/quick_parity.py > $O/parity_$v.txt 2>&1; then
    echo "PARITY FAIL $v"; tail -5 $O/parity_$v.txt; cp /tmp/lib_product.so $L; exit 1
  fi
  echo "parity ok $v"
done
cp /tmp/lib_product.so $L
bash scripts/ab/ab.sh $1 "$3" ${4:-2}
