#!/bin/bash
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r04f; mkdir -p $O
for spec in "coac 1024" "coac 256" "selfplay 8192" "selfplay 1024" "mixed 8192"; do
  set -- $spec
  timeout -k 10 240 python -u scripts/stamps_run.py --workload $1 --envs-per-gpu $2 --steps 30 --json $O/st_$1_$2.json > $O/st_$1_$2.txt 2>&1
done
