#!/bin/bash
# Round 5: phase stamps of configs[1] (1024 envs vs coacAI) with and without the
# speculative batched path finding (translate = stamp 11 -> 12).
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r05g; mkdir -p $O
for v in stamps_old stamps_new; do
  timeout -k 10 300 python scripts/stamps_run.py --workload coac --envs-per-gpu 1024 --steps 30 --lib scripts/ab/libs/$v.so --json $O/$v.json > $O/$v.txt 2>&1
  grep -E "translate|bot_total|end |logic|behaviours|bot_setup" $O/$v.txt
done
