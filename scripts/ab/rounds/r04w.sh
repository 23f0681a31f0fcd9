#!/bin/bash
# Sampler source-row loop: 4 rows per trip with duplicate loads (prev) / 2 rows / 4 and 8 rows without duplicates.
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r04w; mkdir -p $O
bash scripts/ab/ab_bench.sh $O/selfplay 2 "--steps 200 --warmup 30" scripts/ab/libs/prev.so scripts/ab/libs/r2.so scripts/ab/libs/r4n.so scripts/ab/libs/r8n.so
bash scripts/ab/ab_bench.sh $O/coac1024 1 "--workload coac --envs-per-gpu 1024 --steps 300 --warmup 30" scripts/ab/libs/prev.so scripts/ab/libs/r2.so scripts/ab/libs/r4n.so scripts/ab/libs/r8n.so
