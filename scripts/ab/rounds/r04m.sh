#!/bin/bash
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r04m; mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 280 --timeout-method thread -m gpu tests > $O/pytest.txt 2>&1 || { tail -30 $O/pytest.txt; exit 1; }
tail -1 $O/pytest.txt
bash scripts/ab/ab_bench.sh $O/mixed 2 "--workload mixed --steps 200 --warmup 30" scripts/ab/libs/prev.so cur
bash scripts/ab/ab_bench.sh $O/w24 2 "--workload 24x24 --steps 100 --warmup 20" scripts/ab/libs/prev.so cur
timeout -k 10 240 python -u scripts/stamps_run.py --workload 24x24 --envs-per-gpu 8192 --steps 6 --json $O/st_24.json > $O/st_24.txt 2>&1
