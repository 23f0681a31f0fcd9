#!/bin/bash
# Round 5: the sampler's floor in situ (variants that skip the mask-row reads, and
# the source-word read too -- timing only, their picks are wrong), then the full GPU
# suite on the product build.
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r05c; mkdir -p $O
bash scripts/ab/ab_bench.sh $O/selfplay 2 "--steps 200 --warmup 30" cur scripts/ab/libs/floor_nomask.so scripts/ab/libs/floor_storeonly.so
timeout -k 10 1000 python -u -m pytest -x -v --timeout 600 --timeout-method thread -m gpu tests > $O/pytest_gpu.txt 2>&1 || { tail -40 $O/pytest_gpu.txt; exit 1; }
tail -1 $O/pytest_gpu.txt
