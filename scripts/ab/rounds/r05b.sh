#!/bin/bash
# Round 5: the two-groups-per-wave source sampler -- sampler parity tests, then A/B
# against the round-4 library (prev) on the headline and configs[1].
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r05b; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_shard.py -k "sampler" > $O/pytest_sampler.txt 2>&1 || { tail -40 $O/pytest_sampler.txt; exit 1; }
tail -1 $O/pytest_sampler.txt
bash scripts/ab/ab_bench.sh $O/selfplay 3 "--steps 200 --warmup 30" scripts/ab/libs/prev.so cur
bash scripts/ab/ab_bench.sh $O/coac1024 2 "--workload coac --envs-per-gpu 1024 --steps 300 --warmup 30" scripts/ab/libs/prev.so cur
