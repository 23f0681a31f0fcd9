#!/bin/bash
# One gpurun call: GPU parity tests, the bench line, a rocprofv3 kernel-trace
# summary of the same bench command, and separate PMC passes for HBM bytes
# (FETCH_SIZE and WRITE_SIZE cannot share a pass on gfx950).
#   /usr/local/graft/bin/gpurun --timeout 1200 -- bash scripts/gpu_profile.sh TAG
set -euo pipefail
TAG=${1:-run}
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/$TAG
mkdir -p "$O"
BENCH="bench.py --steps 100 --warmup 20 --no-cpu-baseline"
if [ "${SKIP_TESTS:-0}" != 1 ]; then
  timeout -k 10 400 python -m pytest tests -m gpu -x -q > "$O/pytest_gpu.log" 2>&1
fi
timeout -k 10 300 python bench.py > "$O/bench.json" 2> "$O/bench.err"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d "$O/kt" -o kt -- python3 $BENCH > "$O/bench_kt.json" 2> "$O/kt.err"
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -f csv -d "$O/fetch" -o fetch -- python3 $BENCH --no-kernel-events > "$O/bench_fetch.json" 2> "$O/fetch.err"
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -f csv -d "$O/write" -o write -- python3 $BENCH --no-kernel-events > "$O/bench_write.json" 2> "$O/write.err"
# configs[1] (1024 envs vs device coacAI): the kernel trace of its bench command too
COAC="bench.py --workload coac --envs-per-gpu 1024 --steps 300 --warmup 20 --no-cpu-baseline"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d "$O/kt_coac" -o kt -- python3 $COAC > "$O/bench_coac_kt.json" 2> "$O/kt_coac.err"
echo done > "$O/DONE"
