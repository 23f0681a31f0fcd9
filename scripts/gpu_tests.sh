#!/bin/bash
# One gpurun call: the -m gpu suite (optionally a -k filter) and the bench line.
#   /usr/local/graft/bin/gpurun --timeout 1200 -- bash scripts/gpu_tests.sh TAG [-k EXPR]
set -euo pipefail
TAG=${1:-run}
shift || true
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/$TAG
mkdir -p "$O"
timeout -k 10 900 python -m pytest tests -m gpu -q --maxfail=10 "$@" > "$O/pytest_gpu.log" 2>&1 || { echo "pytest failed"; tail -50 "$O/pytest_gpu.log"; exit 1; }
tail -3 "$O/pytest_gpu.log"
timeout -k 10 300 python bench.py > "$O/bench.json" 2> "$O/bench.err"
cat "$O/bench.json"
