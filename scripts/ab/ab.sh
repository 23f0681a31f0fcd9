#!/bin/bash
# experiment A/B: ab.sh TAG "libA libB ..." [rounds] -- interleaved bench runs (coac 1024 + headline) per lib,
# then the stamp runner for every lib*_stamp.so in the list
set -euo pipefail
cd "${GRAFT_REPO_ROOT}"
O=gpurun_out/$1; mkdir -p $O
L=microrts-py_amd/gym_microrts/libmicrorts_amd.so
cp $L /tmp/lib_product.so
for round in $(seq 1 ${3:-2}); do
  for v in $2; do
    cp scripts/ab/lib$v.so $L
    case $v in
      *_stamp) timeout -k 10 300 python scripts/ab/stamps_runner.py 1024 coacAI > $O/stamps_$v.$round.txt 2>&1; echo "$v $round $(head -3 $O/stamps_$v.$round.txt | tail -1)";;
      *)
        timeout -k 10 200 python bench.py --workload coac --envs-per-gpu 1024 --no-cpu-baseline --steps 300 > $O/coac_$v.$round.json 2>/dev/null
        timeout -k 10 200 python bench.py --no-cpu-baseline --steps 150 > $O/head_$v.$round.json 2>/dev/null
        echo "$v $round coac $(python -c "import json; d=json.load(open('$O/coac_$v.$round.json')); print(d['value'], round(d['kernels']['step']['avg_ms']*1000,1))") head $(python -c "import json; d=json.load(open('$O/head_$v.$round.json')); print(d['value'], round(d['kernels']['step']['avg_ms']*1000,1))")";;
    esac
  done
done
cp /tmp/lib_product.so $L
