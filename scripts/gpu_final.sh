#!/bin/bash
# One gpurun call at the round's final build: the -m gpu suite, smoke(), then
# gpu_profile.sh (bench lines, kernel traces, FETCH/WRITE PMC of the headline,
# configs[1] and configs[4], stamped pmc_latest.json) and gpu_sq.sh (SQ occupancy /
# wait / LDS counters of the headline and configs[1]).
#   /usr/local/graft/bin/gpurun --timeout 1200 -- bash scripts/gpu_final.sh TAG
set -euo pipefail
TAG=${1:-final}
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/$TAG
mkdir -p "$O"
timeout -k 10 800 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread --durations=40 > "$O/pytest_gpu.log" 2>&1 \
  || { echo "pytest failed"; tail -40 "$O/pytest_gpu.log"; exit 1; }
tail -1 "$O/pytest_gpu.log"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.log" 2>&1 || { echo "smoke failed"; tail -20 "$O/smoke.log"; exit 1; }
tail -1 "$O/smoke.log"
SKIP_TESTS=1 bash scripts/gpu_profile.sh "$TAG"
bash scripts/gpu_sq.sh "$TAG"
