#!/bin/bash
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r04c; mkdir -p $O
timeout -k 10 300 python scripts/stamps_run.py --workload coac --envs-per-gpu 1024 --steps 40 --json $O/coac1024.json > $O/coac1024.txt 2>&1
timeout -k 10 300 python scripts/stamps_run.py --workload mixed --envs-per-gpu 8192 --steps 20 --json $O/mixed.json > $O/mixed.txt 2>&1
timeout -k 10 300 python scripts/stamps_run.py --workload selfplay --envs-per-gpu 8192 --steps 20 --json $O/selfplay.json > $O/selfplay.txt 2>&1
timeout -k 10 300 python scripts/stamps_run.py --workload partial_obs --envs-per-gpu 4096 --steps 20 --json $O/po.json > $O/po.txt 2>&1
