#!/bin/bash
# One gpurun call: optional GPU tests (PYTEST="files / -k args"), then bench lines
# (BENCHES = ';'-separated bench.py argument lists), each step under its own limit.
#   PYTEST="tests/test_gpu_jni_client.py" BENCHES="--api numpy --steps 20;--workload coac" \
#   /usr/local/graft/bin/gpurun --timeout 900 -- bash scripts/gpu_run.sh TAG
set -euo pipefail
TAG=${1:-run}
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/$TAG
mkdir -p "$O"
if [ -n "${PYTEST:-}" ]; then
  timeout -k 10 ${PYTEST_TIMEOUT:-600} python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu $PYTEST \
    > "$O/pytest_gpu.log" 2>&1 || { echo "pytest failed"; tail -40 "$O/pytest_gpu.log"; exit 1; }
  tail -2 "$O/pytest_gpu.log"
fi
i=0
IFS=';' read -ra B <<< "${BENCHES:-}"
for args in "${B[@]}"; do
  [ -z "$args" ] && continue
  timeout -k 10 ${BENCH_TIMEOUT:-300} python bench.py $args > "$O/bench_$i.json" 2> "$O/bench_$i.err"
  echo "bench $i ($args): $(python -c "import json,sys; d=json.load(open('$O/bench_$i.json')); print(d['value'], d['ms_per_step'], (d.get('roofline') or {}).get('frac'), (d.get('cpu_baseline') or {}).get('value'))")"
  i=$((i+1))
done
echo done > "$O/DONE"
