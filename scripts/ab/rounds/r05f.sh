#!/bin/bash
# Round 5: speculative batched path finding in translateActions (pf_batch + the
# shortest-path lower-bound check): the bot / full-size / policy GPU tests, then A/B vs
# HEAD (prev) on configs[1] (1024 envs vs coacAI), coacAI 8192 and configs[4].
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r05f; mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread -m gpu tests/test_gpu_bots.py tests/test_gpu_policy.py tests/test_gpu_fullsize.py tests/test_gpu_produce_budget.py -k "not 2000_tick and not headline and not selfplay_8192 and not partial_obs" > $O/pytest_bots.txt 2>&1 || { tail -40 $O/pytest_bots.txt; exit 1; }
tail -1 $O/pytest_bots.txt
bash scripts/ab/ab_bench.sh $O/coac1024 3 "--workload coac --envs-per-gpu 1024 --steps 300 --warmup 30" scripts/ab/libs/prev.so cur
bash scripts/ab/ab_bench.sh $O/coac8192 2 "--workload coac --steps 200 --warmup 30" scripts/ab/libs/prev.so cur
bash scripts/ab/ab_bench.sh $O/mixed 2 "--workload mixed --steps 200 --warmup 30" scripts/ab/libs/prev.so cur
