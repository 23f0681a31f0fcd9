#!/bin/bash
# One gpurun call: the -m gpu suite and smoke() on the build in the tree.
#   /usr/local/graft/bin/gpurun --timeout 1200 -- bash scripts/gpu_tests.sh TAG
set -euo pipefail
TAG=${1:-tests}
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/$TAG
mkdir -p "$O"
sha256sum microrts-py_amd/gym_microrts/libmicrorts_amd.so > "$O/lib.sha256"
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread --durations=40 > "$O/pytest_gpu.log" 2>&1 \
  || { echo "pytest failed"; tail -40 "$O/pytest_gpu.log"; exit 1; }
tail -1 "$O/pytest_gpu.log"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.log" 2>&1 || { echo "smoke failed"; tail -20 "$O/smoke.log"; exit 1; }
tail -1 "$O/smoke.log"
