#!/bin/bash
# Round-6 soaks of the bench's own float32-obs kernels against the oracle:
# the 8192-env headline for 10,000 ticks, configs[3]'s 4096 partial-obs envs for 3,000 and
# configs[4]'s 8192-env mixed batch for 2,000, configs[1]'s 1024 envs vs device coacAI for 6,000 --
# every test's obs bit-compared as 1.0f / +0.0f.
#   /usr/local/graft/bin/gpurun --timeout 1200 -- bash scripts/gpu_soak_float.sh TAG [WHICH]
# WHICH: any of headline,partial,mixed,coac (default all).  A heartbeat file under gpurun_out/ keeps
# the silent minutes of one long test from reading as a hang.
set -euo pipefail
TAG=${1:-soak_float}
WHICH=${2:-headline,partial,mixed,coac}
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/$TAG
mkdir -p "$O"
sha256sum microrts-py_amd/gym_microrts/libmicrorts_amd.so > "$O/lib.sha256"
( while true; do sleep 45; date +%T >> "$O/heartbeat.txt"; done ) &
HB=$!
trap 'kill $HB 2>/dev/null || true' EXIT
run() {   # name ticks test-id
  MRTS_SOAK_TICKS=$2 timeout -k 10 $4 python -u -m pytest "$3" -x -v --timeout $(($4 - 20)) --timeout-method thread \
    > "$O/pytest_$1_$2_ticks.log" 2>&1 || { echo "$1 failed"; tail -30 "$O/pytest_$1_$2_ticks.log"; exit 1; }
  tail -1 "$O/pytest_$1_$2_ticks.log"
}
[[ $WHICH == *headline* ]] && run headline_float32 10000 "tests/test_gpu_fullsize.py::test_fullsize_headline_8192_staggered_2000_ticks[float32]" 420
[[ $WHICH == *partial* ]] && run partial_obs4096_float32 3000 "tests/test_gpu_fullsize.py::test_fullsize_partial_obs_4096[float32]" 520
[[ $WHICH == *mixed* ]] && run mixed8192_float32 2000 "tests/test_gpu_fullsize.py::test_fullsize_mixed_buckets_bench_split_8192[float32]" 300
[[ $WHICH == *coac* ]] && run coac1024_float32 6000 "tests/test_gpu_fullsize.py::test_fullsize_coacai_1024" 420
true
