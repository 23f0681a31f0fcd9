#!/bin/bash
# Sampler: source rows per round trip 4 (prev) / 8 (cur) / 16: full GPU suite, then A/B.
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r04v; mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 280 --timeout-method thread tests -m gpu > $O/pytest.txt 2>&1 || { tail -30 $O/pytest.txt; exit 1; }
tail -1 $O/pytest.txt
bash scripts/ab/ab_bench.sh $O/selfplay 3 "--steps 200 --warmup 30" scripts/ab/libs/prev.so cur scripts/ab/libs/rows16.so
bash scripts/ab/ab_bench.sh $O/coac1024 2 "--workload coac --envs-per-gpu 1024 --steps 300 --warmup 30" scripts/ab/libs/prev.so cur scripts/ab/libs/rows16.so
