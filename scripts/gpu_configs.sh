#!/bin/bash
# One gpurun call: the headline bench line plus every secondary BASELINE.json config.
#   /usr/local/graft/bin/gpurun --timeout 1200 -- bash scripts/gpu_configs.sh TAG
set -euo pipefail
TAG=${1:-run}
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/$TAG
mkdir -p "$O"
timeout -k 10 300 python bench.py > "$O/selfplay.json" 2> "$O/selfplay.err"
for spec in "coac 1024" "coac 8192" "workerrush 8192" "partial_obs 4096" "partial_obs 8192" "mixed 8192" "8x8 8192" "24x24 8192"; do
  set -- $spec
  timeout -k 10 300 python bench.py --workload "$1" --envs-per-gpu "$2" --steps 200 --warmup 30 > "$O/$1_$2.json" 2> "$O/$1_$2.err"
done
cat "$O"/*.json
