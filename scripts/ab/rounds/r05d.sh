#!/bin/bash
# Round 5: step kernel at 8 waves / SIMD (amdgpu_waves_per_eu(8, 8): 64 VGPRs, a few spills)
# vs the product's 7, on configs[3]'s 4096 partial-obs envs (2048 games = 1.14 rounds at 7
# workgroups / CU, one round at 8) and the headline.
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r05d; mkdir -p $O
bash scripts/ab/ab_bench.sh $O/partial_obs 3 "--workload partial_obs --envs-per-gpu 4096 --steps 300 --warmup 30" cur scripts/ab/libs/wpe8.so
bash scripts/ab/ab_bench.sh $O/selfplay 2 "--steps 200 --warmup 30" cur scripts/ab/libs/wpe8.so
