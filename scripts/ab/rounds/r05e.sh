#!/bin/bash
# Round 5: masks first in bot-free workgroups (mask words -> mask stream issued -> sight
# disks + one-hot words -> obs stream): full GPU suite, then A/B vs HEAD (prev) on the
# headline and configs[3]'s 4096 partial-obs envs.
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r05e; mkdir -p $O
timeout -k 10 1000 python -u -m pytest -x -q --timeout 600 --timeout-method thread -m gpu tests > $O/pytest_gpu.txt 2>&1 || { tail -40 $O/pytest_gpu.txt; exit 1; }
tail -1 $O/pytest_gpu.txt
bash scripts/ab/ab_bench.sh $O/selfplay 3 "--steps 200 --warmup 30" scripts/ab/libs/prev.so cur
bash scripts/ab/ab_bench.sh $O/partial_obs 3 "--workload partial_obs --envs-per-gpu 4096 --steps 300 --warmup 30" scripts/ab/libs/prev.so cur
