#!/bin/bash
# A/B (experiment libraries, 16x16 / 29 planes / float obs):
#   base = round-3 product; phx = + k_sample_src draws each row's Philox words while its
#   source word / mask rows load; bar = phx + k_step with ~10 fewer workgroup barriers per tick
# bit-exact checks on phx / bar first (sampler GPU tests, quick_parity), then interleaved
# headline and configs[1] benches.
set -euo pipefail
cd "${GRAFT_REPO_ROOT}"
O=gpurun_out/${1:-phx}; mkdir -p $O
L=microrts-py_amd/gym_microrts/libmicrorts_amd.so
cp $L /tmp/lib_product.so
restore() { cp /tmp/lib_product.so $L; }
trap restore EXIT
cp scripts/ab/libbar.so $L
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_shard.py -k sampler -x -v --timeout 200 --timeout-method thread > $O/pytest_sampler.log 2>&1 \
  || { echo "pytest failed"; tail -30 $O/pytest_sampler.log; exit 1; }
tail -1 $O/pytest_sampler.log
timeout -k 10 400 python scripts/ab/quick_parity.py > $O/parity_bar.log 2>&1 || { echo "parity FAILED bar"; tail -8 $O/parity_bar.log; exit 1; }
echo "parity ok bar"
for round in 1 2 3; do
  for v in base phx bar; do
    cp scripts/ab/lib$v.so $L
    timeout -k 10 200 python bench.py --no-cpu-baseline --steps 150 > $O/head_$v.$round.json 2>/dev/null
    timeout -k 10 200 python bench.py --no-cpu-baseline --workload coac --envs-per-gpu 1024 --steps 300 > $O/coac_$v.$round.json 2>/dev/null
    echo "$v $round head $(python -c "import json; d=json.load(open('$O/head_$v.$round.json')); print(d['value'], round(d['kernels']['step']['avg_ms']*1000,1), round(d['kernels']['sample']['avg_ms']*1000,1))") coac $(python -c "import json; d=json.load(open('$O/coac_$v.$round.json')); print(d['value'], round(d['kernels']['step']['avg_ms']*1000,1), round(d['kernels']['sample']['avg_ms']*1000,1))")"
  done
done
echo done > $O/DONE
