#!/bin/bash
# One gpurun call at a build: the -m gpu suite, the bench line, rocprofv3
# kernel-trace summaries and separate PMC passes (FETCH_SIZE and WRITE_SIZE cannot
# share a pass on gfx950) of the headline and of configs[1] (1024 envs vs device
# coacAI).  The PMC summary is stamped with the library's sha256 and copied to
# profiles/pmc_latest.json on the box, so the final bench lines carry traffic.
#   /usr/local/graft/bin/gpurun --timeout 1200 -- bash scripts/gpu_profile.sh TAG
#   SKIP_TESTS=1 to skip the suite.
set -euo pipefail
TAG=${1:-run}
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/$TAG
mkdir -p "$O"
if [ "${SKIP_TESTS:-0}" != 1 ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > "$O/pytest_gpu.log" 2>&1 \
    || { echo "pytest failed"; tail -40 "$O/pytest_gpu.log"; exit 1; }
  tail -2 "$O/pytest_gpu.log"
fi
BENCH="bench.py --steps 100 --warmup 20 --no-cpu-baseline"
COAC="bench.py --workload coac --envs-per-gpu 1024 --steps 300 --warmup 20 --no-cpu-baseline"
MIXED="bench.py --workload mixed --steps 100 --warmup 20 --no-cpu-baseline"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d "$O/kt" -o kt -- python3 $BENCH > "$O/bench_kt.json" 2> "$O/kt.err"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d "$O/kt_coac" -o kt -- python3 $COAC > "$O/bench_coac_kt.json" 2> "$O/kt_coac.err"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d "$O/kt_mixed" -o kt -- python3 $MIXED > "$O/bench_mixed_kt.json" 2> "$O/kt_mixed.err"
for W in selfplay coac mixed; do
  case $W in
    selfplay) CMD="$BENCH"; KEY=selfplay@8192;;
    coac) CMD="$COAC"; KEY=coac@1024;;
    mixed) CMD="$MIXED"; KEY=mixed@8192;;
  esac
  timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE -f csv -d "$O/pmc_$W/fetch" -o fetch -- python3 $CMD --no-kernel-events > "$O/pmc_$W.fetch.json" 2> "$O/pmc_$W.fetch.err"
  timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE -f csv -d "$O/pmc_$W/write" -o write -- python3 $CMD --no-kernel-events > "$O/pmc_$W.write.json" 2> "$O/pmc_$W.write.err"
  python3 scripts/pmc_summary.py "$O/pmc_$W" "$O/pmc_latest.json" --workload $KEY --command "$CMD" > "$O/pmc_$W.txt"
done
cp "$O/pmc_latest.json" profiles/pmc_latest.json
timeout -k 10 300 python bench.py > "$O/bench.json" 2> "$O/bench.err"
timeout -k 10 300 python bench.py --workload coac --envs-per-gpu 1024 --no-cpu-baseline > "$O/bench_coac.json" 2> "$O/bench_coac.err"
timeout -k 10 300 python bench.py --workload mixed --no-cpu-baseline > "$O/bench_mixed.json" 2> "$O/bench_mixed.err"
cat "$O/bench.json" "$O/bench_coac.json" "$O/bench_mixed.json"
echo done > "$O/DONE"
