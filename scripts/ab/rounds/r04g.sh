#!/bin/bash
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r04g; mkdir -p $O
for K in 0 1; do
  for spec in "coac 1024" "selfplay 8192"; do
    set -- $spec
    HIP_FORCE_DEV_KERNARG=$K timeout -k 10 240 python -u scripts/stamps_run.py --workload $1 --envs-per-gpu $2 --steps 20 --json $O/st_k${K}_$1_$2.json > $O/st_k${K}_$1_$2.txt 2>&1
  done
  HIP_FORCE_DEV_KERNARG=$K timeout -k 10 240 python bench.py --steps 200 --warmup 30 --no-cpu-baseline > $O/bench_k${K}_selfplay.json 2>&1
  HIP_FORCE_DEV_KERNARG=$K timeout -k 10 240 python bench.py --workload coac --envs-per-gpu 1024 --steps 300 --warmup 30 --no-cpu-baseline > $O/bench_k${K}_coac.json 2>&1
done
