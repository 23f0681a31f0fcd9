#!/bin/bash
# A/B: new (HEAD product) vs pb (+ phase-B index math without division: (c, plane) and
# (row, channel) advance by constants, branch-free ch == 76 fix-up) vs pb2 (+ snapshot and
# commute check in one pass, unit counts instead of the post-execution scan, prod compaction
# without its trailing barrier).  quick_parity on the candidates first.
set -euo pipefail
cd "${GRAFT_REPO_ROOT}"
O=gpurun_out/${1:-pb}; mkdir -p $O
L=microrts-py_amd/gym_microrts/libmicrorts_amd.so
cp $L /tmp/lib_product.so
restore() { cp /tmp/lib_product.so $L; }
trap restore EXIT
for v in ${CANDS:-pb2 cs2}; do
  cp scripts/ab/lib$v.so $L
  timeout -k 10 400 python scripts/ab/quick_parity.py > $O/parity_$v.log 2>&1 || { echo "parity FAILED $v"; tail -8 $O/parity_$v.log; exit 1; }
  echo "parity ok $v"
done
for round in 1 2 3; do
  for v in new ${CANDS:-pb2 cs2}; do
    cp scripts/ab/lib$v.so $L
    timeout -k 10 200 python bench.py --no-cpu-baseline --steps 150 > $O/head_$v.$round.json 2>/dev/null
    timeout -k 10 200 python bench.py --no-cpu-baseline --workload coac --envs-per-gpu 1024 --steps 300 > $O/coac_$v.$round.json 2>/dev/null
    echo "$v $round head $(python -c "import json; d=json.load(open('$O/head_$v.$round.json')); print(d['value'], round(d['kernels']['step']['avg_ms']*1000,1), round(d['kernels']['sample']['avg_ms']*1000,1))") coac $(python -c "import json; d=json.load(open('$O/coac_$v.$round.json')); print(d['value'], round(d['kernels']['step']['avg_ms']*1000,1), round(d['kernels']['sample']['avg_ms']*1000,1))")"
  done
done
echo done > $O/DONE
