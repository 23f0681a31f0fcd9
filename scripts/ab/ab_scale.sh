#!/bin/bash
# ab_scale.sh TAG "libs" rounds -- headline k_step time at 512 / 2048 / 8192 envs, plus coac 1024, per lib
set -euo pipefail
cd "${GRAFT_REPO_ROOT}"
O=gpurun_out/$1; mkdir -p $O
L=microrts-py_amd/gym_microrts/libmicrorts_amd.so
cp $L /tmp/lib_product.so
for round in $(seq 1 $3); do
  for v in $2; do
    cp scripts/ab/lib$v.so $L
    line="$v $round"
    for n in 512 2048 8192; do
      timeout -k 10 200 python bench.py --no-cpu-baseline --steps 150 --envs-per-gpu $n > $O/head_${v}_$n.$round.json 2>/dev/null
      line="$line | $n: $(python -c "import json; d=json.load(open('$O/head_${v}_$n.$round.json')); print(round(d['kernels']['step']['avg_ms']*1000,1))")"
    done
    timeout -k 10 200 python bench.py --workload coac --envs-per-gpu 1024 --no-cpu-baseline --steps 300 > $O/coac_$v.$round.json 2>/dev/null
    line="$line | coac1024: $(python -c "import json; d=json.load(open('$O/coac_$v.$round.json')); print(round(d['kernels']['step']['avg_ms']*1000,1))")"
    echo "$line"
  done
done
cp /tmp/lib_product.so $L
