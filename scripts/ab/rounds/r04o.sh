#!/bin/bash
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r04o; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 280 --timeout-method thread tests/test_gpu_shard.py tests/test_gpu_parity.py tests/test_gpu_fullsize.py -k "sampler or headline or shard or offset" > $O/pytest.txt 2>&1 || { tail -30 $O/pytest.txt; exit 1; }
tail -1 $O/pytest.txt
bash scripts/ab/ab_bench.sh $O/selfplay 3 "--steps 200 --warmup 30" scripts/ab/libs/prev.so cur
bash scripts/ab/ab_bench.sh $O/coac1024 2 "--workload coac --envs-per-gpu 1024 --steps 300 --warmup 30" scripts/ab/libs/prev.so cur
