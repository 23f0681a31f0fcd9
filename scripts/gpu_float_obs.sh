#!/bin/bash
# the float32-obs lock-steps (the bench's own kernels) on the MI355X,
# then the headline float32 lock-step once more under rocprofv3 --kernel-trace, whose
# kernel list must show k_step<256, 29, float, false>.
#   /usr/local/graft/bin/gpurun --timeout 1200 -- bash scripts/gpu_float_obs.sh TAG
set -euo pipefail
TAG=${1:-float_obs}
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/$TAG
mkdir -p "$O"
export TMPDIR=/tmp
sha256sum microrts-py_amd/gym_microrts/libmicrorts_amd.so > "$O/lib.sha256"
timeout -k 10 700 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -m gpu -x -v \
  -k "float32 or obs_dtype or fullsize" --timeout 600 --timeout-method thread --durations=0 > "$O/pytest_float.log" 2>&1 \
  || { echo "pytest failed"; tail -40 "$O/pytest_float.log"; exit 1; }
tail -1 "$O/pytest_float.log"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -f csv -d "$O/prof" -o headline -- python -u -m pytest \
  "tests/test_gpu_fullsize.py::test_fullsize_headline_8192_staggered_2000_ticks[float32]" -x -q --timeout 350 \
  --timeout-method thread > "$O/rocprof_headline.log" 2>&1 || { echo "rocprof run failed"; tail -30 "$O/rocprof_headline.log"; exit 1; }
tail -1 "$O/rocprof_headline.log"
find "$O/prof" -name "*kernel_stats.csv" | head -1 | xargs -I{} cp {} "$O/headline_kernel_stats.csv"
cut -d, -f1-4 "$O/headline_kernel_stats.csv" | head -20
