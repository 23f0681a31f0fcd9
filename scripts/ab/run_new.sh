#!/bin/bash
# The product build at HEAD (sampler Philox overlap + fewer k_step barriers): the whole -m gpu
# suite, then interleaved A/B vs the round-3 product (base) on the headline and configs[1].
set -euo pipefail
cd "${GRAFT_REPO_ROOT}"
O=gpurun_out/${1:-new}; mkdir -p $O
L=microrts-py_amd/gym_microrts/libmicrorts_amd.so
cp $L /tmp/lib_product.so
restore() { cp /tmp/lib_product.so $L; }
trap restore EXIT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > $O/pytest_gpu.log 2>&1 \
  || { echo "pytest failed"; tail -40 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
for round in 1 2 3; do
  for v in base new; do
    cp scripts/ab/lib$v.so $L
    timeout -k 10 200 python bench.py --no-cpu-baseline --steps 150 > $O/head_$v.$round.json 2>/dev/null
    timeout -k 10 200 python bench.py --no-cpu-baseline --workload coac --envs-per-gpu 1024 --steps 300 > $O/coac_$v.$round.json 2>/dev/null
    echo "$v $round head $(python -c "import json; d=json.load(open('$O/head_$v.$round.json')); print(d['value'], round(d['kernels']['step']['avg_ms']*1000,1), round(d['kernels']['sample']['avg_ms']*1000,1))") coac $(python -c "import json; d=json.load(open('$O/coac_$v.$round.json')); print(d['value'], round(d['kernels']['step']['avg_ms']*1000,1), round(d['kernels']['sample']['avg_ms']*1000,1))")"
  done
done
echo done > $O/DONE
