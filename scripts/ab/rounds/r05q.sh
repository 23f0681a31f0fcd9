#!/bin/bash
# Round 5: the fused bot wave's id read with the game state instead of where the bot starts
# (there its load's s_waitcnt vmcnt(0) also waited for the wave's own state write-back and
# reward stores).  Same-box interleaved A/B on configs[1] (1024 envs vs coacAI), coacAI at
# 8192 and the headline; base = HEAD before the change, aipf = the id held in a VGPR,
# aipf2 = the id parked in LDS (the early counter's spare word).
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r05q2
L="scripts/ab/libs/base.so scripts/ab/libs/aipf.so scripts/ab/libs/aipf2.so"
bash scripts/ab/ab_bench.sh $O/coac1024 4 "--workload coac --envs-per-gpu 1024 --steps 300 --warmup 30" $L
bash scripts/ab/ab_bench.sh $O/coac8192 2 "--workload coac --envs-per-gpu 8192 --steps 100 --warmup 20" $L
bash scripts/ab/ab_bench.sh $O/workerrush8192 2 "--workload workerrush --envs-per-gpu 8192 --steps 100 --warmup 20" $L
bash scripts/ab/ab_bench.sh $O/selfplay 2 "--steps 100 --warmup 20" $L
