#!/bin/bash
# One gpurun call: the bot GPU tests and the bot workloads with / without the
# bot fusion (mrts_set_bot_fusion).
#   /usr/local/graft/bin/gpurun --timeout 1200 -- bash scripts/gpu_bots_ab.sh TAG
set -euo pipefail
TAG=${1:-bots}
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/$TAG
mkdir -p "$O"
timeout -k 10 240 python -c 'import __graft_entry__ as g; g.smoke(); print("smoke ok")' > "$O/smoke.log" 2>&1 || { cat "$O/smoke.log"; exit 1; }
timeout -k 10 600 python -u -m pytest tests/test_gpu_bots.py tests/test_driver_compat.py tests/test_capi.py tests/test_gpu_fullsize.py tests/test_gpu_sharedmem.py -m gpu -x -q \
  --timeout 300 --timeout-method thread > "$O/pytest_bots.log" 2>&1 || { tail -40 "$O/pytest_bots.log"; exit 1; }
tail -2 "$O/pytest_bots.log"
for spec in "coac 1024" "coac 8192" "workerrush 8192" "mixed 8192"; do
  set -- $spec
  timeout -k 10 300 python bench.py --workload "$1" --envs-per-gpu "$2" --steps 200 --warmup 30 --no-cpu-baseline --bot-fusion 0 > "$O/$1_$2_unfused.json" 2> "$O/$1_$2_unfused.err"
  timeout -k 10 300 python bench.py --workload "$1" --envs-per-gpu "$2" --steps 200 --warmup 30 --no-cpu-baseline > "$O/$1_$2.json" 2> "$O/$1_$2.err"
done
for f in "$O"/*.json; do python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[1].split('/')[-1], round(d['value']/1e6,2), 'M', d.get('kernels'))" "$f"; done
