#!/bin/bash
# ab_wl.sh TAG "libs" rounds "workload:envs ..." -- interleaved bench step-kernel times per workload
set -euo pipefail
cd "${GRAFT_REPO_ROOT}"
O=gpurun_out/$1; mkdir -p $O
L=microrts-py_amd/gym_microrts/libmicrorts_amd.so
cp $L /tmp/lib_product.so
for round in $(seq 1 $3); do
  for v in $2; do
    cp scripts/ab/lib$v.so $L
    line="$v $round"
    for wl in $4; do
      w=${wl%%:*}; n=${wl##*:}
      timeout -k 10 200 python bench.py --no-cpu-baseline --steps 150 --workload $w --envs-per-gpu $n > $O/${v}_${w}_$n.$round.json 2>/dev/null
      line="$line | $w@$n: $(python -c "import json; d=json.load(open('$O/${v}_${w}_$n.$round.json')); print(d['value'], round(d['roofline']['avg_launch_ms']*1000,1))")"
    done
    echo "$line"
  done
done
cp /tmp/lib_product.so $L
