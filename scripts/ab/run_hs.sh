#!/bin/bash
set -euo pipefail
cd "${GRAFT_REPO_ROOT}"
O=gpurun_out/hs; mkdir -p $O
L=microrts-py_amd/gym_microrts/libmicrorts_amd.so
cp $L /tmp/lib_product.so
cp scripts/ab/libcur_headstamp.so $L
for n in 512 2048 8192; do
  timeout -k 10 300 python scripts/ab/stamps_head.py $n > $O/headstamps_$n.json 2> $O/headstamps_$n.err
  python -c "import json; d=json.load(open('$O/headstamps_$n.json')); print($n, {k: v for k, v in d.items() if not isinstance(v, list)})"
done
cp /tmp/lib_product.so $L
