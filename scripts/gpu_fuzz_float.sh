#!/bin/bash
# Round-6 campaigns with the float32-obs arms (odd fuzz seeds, k % 4 >= 2 of the reference-generator
# maps, odd random-map seeds, the boundary shapes' k_bot arm): the bench's dtype compared as bits
# against the oracle's one-hot on every engine surface the fuzzers reach.
#   /usr/local/graft/bin/gpurun --timeout 1200 -- bash scripts/gpu_fuzz_float.sh TAG [SEEDS [FIRST [PARTS]]]
# PARTS: any of fuzz,pcg,random,checkpoint (default fuzz,pcg,random)
set -euo pipefail
TAG=${1:-fuzz_float}
SEEDS=${2:-800}
FIRST=${3:-0}
PARTS=${4:-fuzz,pcg,random}
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/$TAG
mkdir -p "$O"
sha256sum microrts-py_amd/gym_microrts/libmicrorts_amd.so > "$O/lib.sha256"
( while true; do sleep 45; date +%T >> "$O/heartbeat.txt"; done ) &
HB=$!
trap 'kill $HB 2>/dev/null || true' EXIT
step() {  # name seconds VAR=value pytest-args...
  local name=$1 secs=$2 var=$3; shift 3
  env "$var" MRTS_FUZZ_FIRST=$FIRST timeout -k 10 "$secs" python -u -m pytest "$@" -m gpu -x -v --timeout 280 --timeout-method thread \
    > "$O/pytest_$name.log" 2>&1 || { echo "$name failed"; tail -40 "$O/pytest_$name.log"; exit 1; }
  tail -1 "$O/pytest_$name.log"
}
[[ $PARTS == *fuzz* ]] && step fuzz 420 MRTS_FUZZ_SEEDS=$SEEDS tests/test_gpu_fuzz_maps.py -k "fuzz_map_lockstep or step_group or large_map"
[[ $PARTS == *pcg* ]] && step pcg_campaign 300 MRTS_PCG_CAMPAIGN=300 tests/test_pcg_maps.py -k campaign
[[ $PARTS == *random* ]] && step random_and_boundary 300 MRTS_NONE=1 tests/test_gpu_random_maps.py tests/test_max_map_sizes.py
[[ $PARTS == *checkpoint* ]] && step checkpoint 300 MRTS_FUZZ_SEEDS=$SEEDS tests/test_gpu_checkpoint.py -k fuzz
true
