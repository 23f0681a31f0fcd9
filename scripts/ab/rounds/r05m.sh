#!/bin/bash
# Round 5: (1) 24x24 (HW > 256, unfused) step on 512-lane workgroups vs 256;
# (2) configs[4]'s two grouped step launches concurrently (the 24x24 launch on a side
# stream forked from / joined to the caller's; experiment policy bit 8) vs back to back.
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r05m; mkdir -p $O
bash scripts/ab/ab_bench.sh $O/24x24 2 "--workload 24x24 --steps 100 --warmup 20" cur scripts/ab/libs/nt512.so
for r in 1 2 3; do
  bash scripts/ab/ab_bench.sh $O/mixed_r$r 1 "--workload mixed --steps 200 --warmup 30" cur
  bash scripts/ab/ab_bench.sh $O/mixed_r$r 1 "--workload mixed --steps 200 --warmup 30 --group-policy 13" scripts/ab/libs/conc.so
done
