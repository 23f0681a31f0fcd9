#!/bin/bash
# Round 5: configs[1]'s slowest 2 % of games, phase by phase (stamped product build)
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r05h; mkdir -p $O
timeout -k 10 300 python scripts/stamps_run.py --workload coac --envs-per-gpu 1024 --steps 40 --lib scripts/ab/libs/stamps_old.so --json $O/coac_1024.json > $O/coac_1024.txt 2>&1
grep -v amdgpu.ids $O/coac_1024.txt
