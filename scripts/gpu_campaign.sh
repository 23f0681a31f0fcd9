#!/bin/bash
# Round-6 parity campaigns on the MI355X: all 300 reference-generator maps
# (tests/golden/maps/pcg_campaign.json) and random maps of the largest accepted shapes.
#   /usr/local/graft/bin/gpurun --timeout 1200 -- bash scripts/gpu_campaign.sh TAG [LARGE_SEEDS]
set -euo pipefail
TAG=${1:-campaign}
LARGE=${2:-60}
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/$TAG
mkdir -p "$O"
sha256sum microrts-py_amd/gym_microrts/libmicrorts_amd.so > "$O/lib.sha256"
MRTS_PCG_CAMPAIGN=300 timeout -k 10 700 python -u -m pytest tests/test_pcg_maps.py -m gpu -x -v -k campaign \
  --timeout 280 --timeout-method thread > "$O/pytest_pcg_campaign.log" 2>&1 \
  || { echo "pcg campaign failed"; tail -40 "$O/pytest_pcg_campaign.log"; exit 1; }
tail -1 "$O/pytest_pcg_campaign.log"
MRTS_FUZZ_SEEDS=$((LARGE * 6)) timeout -k 10 400 python -u -m pytest tests/test_gpu_fuzz_maps.py -m gpu -x -v -k large \
  --timeout 280 --timeout-method thread > "$O/pytest_large_fuzz.log" 2>&1 \
  || { echo "large fuzz failed"; tail -40 "$O/pytest_large_fuzz.log"; exit 1; }
tail -1 "$O/pytest_large_fuzz.log"
