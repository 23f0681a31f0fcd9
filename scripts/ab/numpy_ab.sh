#!/bin/bash
set -euo pipefail
cd "${GRAFT_REPO_ROOT}"
O=gpurun_out/$1; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_contracts.py tests/test_gpu_sharedmem.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for r in 1 2 3; do
  timeout -k 10 300 python bench.py --api ${API:-numpy} --steps 30 --warmup 5 --no-cpu-baseline > $O/numpy_$r.json 2> $O/numpy_$r.err
  python -c "import json; d=json.load(open('$O/numpy_$r.json')); print('numpy r$r', round(d['value']/1e3,1), 'k', d['ms_per_step'])"
done
