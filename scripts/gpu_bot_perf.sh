#!/bin/bash
# Bot-config throughput (steady state, staggered pre-roll): configs[1] (1024 envs vs coacAI) and the
# 8192-env bot workloads.  One gpurun call:
#   /usr/local/graft/bin/gpurun --timeout 900 -- bash scripts/gpu_bot_perf.sh TAG [pytest -k expr]
set -euo pipefail
TAG=${1:-bots}
K=${2:-}
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/$TAG
mkdir -p "$O"
if [ -n "$K" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -q -x -k "$K" --timeout 300 --timeout-method thread > "$O/pytest.log" 2>&1 \
    || { echo "pytest failed"; tail -30 "$O/pytest.log"; exit 1; }
  tail -2 "$O/pytest.log"
fi
for w in "coac 1024" "coac 8192" "workerrush 8192"; do
  set -- $w
  timeout -k 10 200 python bench.py --workload $1 --envs-per-gpu $2 --no-cpu-baseline > "$O/${1}_$2.json" 2>> "$O/bench.err"
  python -c "import json,sys; d=json.load(open('$O/${1}_$2.json')); print('$1', $2, round(d['value']/1e6,2), 'M/s', 'step', d['kernels']['step']['avg_ms'], 'frac', d['roofline']['frac'])"
done
