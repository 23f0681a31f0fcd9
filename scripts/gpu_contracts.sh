#!/bin/bash
# Host-contract measurements: PCIe probe, the numpy
# contract bench at 8192 envs, and the GridNet PPO driver at configs[3]'s 4096 envs
# (partial obs, ppo_gridnet.py's bot mix) under the numpy / hybrid / tensor contracts.
#   /usr/local/graft/bin/gpurun --timeout 900 -- bash scripts/gpu_contracts.sh TAG
set -euo pipefail
TAG=${1:-contracts}
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/$TAG
mkdir -p "$O"
timeout -k 10 180 python scripts/pcie_probe.py > "$O/pcie.json" 2> "$O/pcie.err"
timeout -k 10 300 python bench.py --api numpy --steps 40 --warmup 5 --preroll 200 --no-cpu-baseline > "$O/bench_numpy.json" 2> "$O/bench_numpy.err"
for API in numpy hybrid tensor; do
  timeout -k 10 300 python examples/ppo_gridnet_driver.py --num-selfplay-envs 4072 --num-bot-envs 24 --partial-obs \
      --num-steps 16 --updates 3 --api $API > "$O/ppo_$API.jsonl" 2> "$O/ppo_$API.err"
done
for f in "$O"/ppo_*.jsonl; do tail -n 1 "$f"; done
echo done > "$O/DONE"
