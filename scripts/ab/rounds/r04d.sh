#!/bin/bash
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r04d; mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 280 --timeout-method thread -m gpu tests > $O/pytest.txt 2>&1 || { tail -30 $O/pytest.txt; exit 1; }
tail -2 $O/pytest.txt
bash scripts/ab/ab_bench.sh $O/coac1024 2 "--workload coac --envs-per-gpu 1024 --steps 300 --warmup 30" scripts/ab/libs/head.so scripts/ab/libs/lds.so cur
bash scripts/ab/ab_bench.sh $O/mixed 2 "--workload mixed --steps 200 --warmup 30" scripts/ab/libs/head.so scripts/ab/libs/lds.so cur scripts/ab/libs/cap6.so
bash scripts/ab/ab_bench.sh $O/coac8192 1 "--workload coac --steps 200 --warmup 30" scripts/ab/libs/head.so cur
bash scripts/ab/ab_bench.sh $O/selfplay 1 "--steps 200 --warmup 30" scripts/ab/libs/head.so cur
timeout -k 10 300 python scripts/stamps_run.py --workload coac --envs-per-gpu 1024 --steps 40 --json $O/st_coac1024.json > $O/st_coac1024.txt 2>&1
timeout -k 10 300 python scripts/stamps_run.py --workload mixed --envs-per-gpu 8192 --steps 20 --json $O/st_mixed.json > $O/st_mixed.txt 2>&1
timeout -k 10 300 python scripts/stamps_run.py --workload selfplay --envs-per-gpu 8192 --steps 20 --json $O/st_selfplay.json > $O/st_selfplay.txt 2>&1
