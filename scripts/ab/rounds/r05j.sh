#!/bin/bash
# Round 5: the sampler walking the rows newest-written first (reversed block order:
# the last games' mask rows, written last by k_step, may still sit in the MALL).
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r05j; mkdir -p $O
bash scripts/ab/ab_bench.sh $O/selfplay 3 "--steps 200 --warmup 30" cur scripts/ab/libs/sampler_rev.so
