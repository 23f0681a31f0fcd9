#!/bin/bash
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r04l; mkdir -p $O
for spec in "mixed 8192" "partial_obs 4096" "24x24 8192"; do
  set -- $spec
  timeout -k 10 240 python -u scripts/stamps_run.py --workload $1 --envs-per-gpu $2 --steps 8 --json $O/st_$1_$2.json > $O/st_$1_$2.txt 2>&1
done
