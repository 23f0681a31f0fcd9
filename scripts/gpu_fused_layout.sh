#!/bin/bash
# One gpurun call: bot GPU tests + bot workloads (fused k_step LDS layout check).
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${1:-fl}
mkdir -p "$O"
timeout -k 10 240 python -c 'import __graft_entry__ as g; g.smoke(); print("smoke ok")' > "$O/smoke.log" 2>&1 || { cat "$O/smoke.log"; exit 1; }
timeout -k 10 600 python -u -m pytest tests/test_gpu_bots.py tests/test_gpu_fullsize.py tests/test_gpu_sharedmem.py -m gpu -x -q \
  --timeout 300 --timeout-method thread > "$O/pytest.log" 2>&1 || { tail -40 "$O/pytest.log"; exit 1; }
tail -2 "$O/pytest.log"
for spec in "coac 1024" "coac 8192" "workerrush 8192" "mixed 8192"; do
  set -- $spec
  timeout -k 10 300 python bench.py --workload "$1" --envs-per-gpu "$2" --steps 200 --warmup 30 --no-cpu-baseline > "$O/$1_$2.json" 2> "$O/$1_$2.err"
done
for f in "$O"/*.json; do python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[1].split('/')[-1], round(d['value']/1e6,2), 'M', {k:round(v['avg_ms']*1e3,1) for k,v in d.get('kernels',{}).items()})" "$f"; done
