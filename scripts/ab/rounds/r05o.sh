#!/bin/bash
# Round 5: translateActions' free-cell / ResourceUsage checks from the bot's row words
# instead of LDS round trips: bot / policy / full-size / produce GPU tests, A/B vs HEAD
# (prev) on configs[1], coacAI 8192 and configs[4], then the stamped counters.
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r05o; mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread -m gpu tests/test_gpu_bots.py tests/test_gpu_policy.py tests/test_gpu_fullsize.py tests/test_gpu_produce_budget.py tests/test_gpu_checkpoint.py -k "not 2000_tick and not headline and not selfplay_8192 and not partial_obs" > $O/pytest_bots.txt 2>&1 || { tail -40 $O/pytest_bots.txt; exit 1; }
tail -1 $O/pytest_bots.txt
bash scripts/ab/ab_bench.sh $O/coac1024 3 "--workload coac --envs-per-gpu 1024 --steps 300 --warmup 30" scripts/ab/libs/prev.so cur
bash scripts/ab/ab_bench.sh $O/coac8192 2 "--workload coac --steps 200 --warmup 30" scripts/ab/libs/prev.so cur
bash scripts/ab/ab_bench.sh $O/mixed 2 "--workload mixed --steps 200 --warmup 30" scripts/ab/libs/prev.so cur
timeout -k 10 300 python scripts/stamps_run.py --workload coac --envs-per-gpu 1024 --steps 40 --lib scripts/ab/libs/stamps.so --json $O/stamps_coac_1024.json > $O/stamps_coac_1024.txt 2>&1
grep -E "translate|slow2_end|slow2_translate|slow2_bot_(entries|searches|search_us)" $O/stamps_coac_1024.txt
