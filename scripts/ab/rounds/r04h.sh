#!/bin/bash
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r04h2; mkdir -p $O
for R in 0 1024; do
  for spec in "coac 1024" "selfplay 8192" "selfplay 2048" "selfplay 4096"; do
    set -- $spec
    timeout -k 10 240 python -u scripts/stamps_run.py --workload $1 --envs-per-gpu $2 --steps 20 --read-mb $R --json $O/st_r${R}_$1_$2.json > $O/st_r${R}_$1_$2.txt 2>&1
  done
done
