#!/bin/bash
# Round 5: configs[4]'s launch plan -- [0,0,1] (8x8 + 16x16, then 24x24: the 24x24 launch's
# 1536 workgroups fill 1.5 rounds of its 4-per-CU slots) vs [0,1,0] (the 8x8 games fill the
# 24x24 launch's second round; 16x16 alone).  Experiment build: -DMRTS_EXP_PLAN.
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r05s
bash scripts/ab/ab_bench.sh $O/mixed 3 "--workload mixed --envs-per-gpu 8192 --steps 200 --warmup 30" scripts/ab/libs/base.so scripts/ab/libs/plan010.so
