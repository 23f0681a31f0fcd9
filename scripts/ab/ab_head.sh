#!/bin/bash
# ab_head.sh TAG "libs" rounds -- interleaved headline bench runs (k_step event time), then headline stamps of *_headstamp libs
set -euo pipefail
cd "${GRAFT_REPO_ROOT}"
O=gpurun_out/$1; mkdir -p $O
L=microrts-py_amd/gym_microrts/libmicrorts_amd.so
cp $L /tmp/lib_product.so
for round in $(seq 1 $3); do
  for v in $2; do
    cp scripts/ab/lib$v.so $L
    case $v in
      *_headstamp) timeout -k 10 300 python scripts/ab/stamps_head.py > $O/headstamps_$v.$round.json 2> /dev/null; echo "$v $round $(python -c "import json; d=json.load(open('$O/headstamps_$v.$round.json')); print(round(d['span_us'],1), d['first_stream_start_us'], d['last_start_us'])")";;
      *) timeout -k 10 200 python bench.py --no-cpu-baseline --steps 150 > $O/head_$v.$round.json 2>/dev/null
         echo "$v $round head $(python -c "import json; d=json.load(open('$O/head_$v.$round.json')); print(d['value'], round(d['kernels']['step']['avg_ms']*1000,1), round(d['kernels']['sample']['avg_ms']*1000,1))")";;
    esac
  done
done
cp /tmp/lib_product.so $L
