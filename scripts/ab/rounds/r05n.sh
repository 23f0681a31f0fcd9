#!/bin/bash
# Round 5: configs[1] bot counters per game (translate entries, path searches, their
# time, four-layer rounds), all games and the slowest 2 %
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r05n; mkdir -p $O
timeout -k 10 300 python scripts/stamps_run.py --workload coac --envs-per-gpu 1024 --steps 40 --lib scripts/ab/libs/stamps.so --json $O/coac_1024.json > $O/coac_1024.txt 2>&1
grep -v amdgpu.ids $O/coac_1024.txt
