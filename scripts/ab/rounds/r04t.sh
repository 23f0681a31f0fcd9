#!/bin/bash
# Bot games: view-0 action rows prefetched with the state: full GPU suite, then A/B vs previous build.
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r04t; mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 280 --timeout-method thread tests -m gpu > $O/pytest.txt 2>&1 || { tail -30 $O/pytest.txt; exit 1; }
tail -1 $O/pytest.txt
bash scripts/ab/ab_bench.sh $O/coac1024 3 "--workload coac --envs-per-gpu 1024 --steps 300 --warmup 30" scripts/ab/libs/prev.so cur
bash scripts/ab/ab_bench.sh $O/selfplay 2 "--steps 200 --warmup 30" scripts/ab/libs/prev.so cur
bash scripts/ab/ab_bench.sh $O/mixed 2 "--workload mixed --steps 100 --warmup 20" scripts/ab/libs/prev.so cur
bash scripts/ab/ab_bench.sh $O/coac8192 2 "--workload coac --envs-per-gpu 8192 --steps 100 --warmup 20" scripts/ab/libs/prev.so cur
