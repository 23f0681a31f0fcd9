#!/bin/bash
set -euo pipefail
cd "${GRAFT_REPO_ROOT}"
O=gpurun_out/$1; mkdir -p $O
for round in 1 2; do
  for m in 0 1; do
    MIXED_CONCURRENT=$m timeout -k 10 300 python scripts/ab/mixed_concurrent.py --workload mixed --no-cpu-baseline --steps 200 --warmup 30 > $O/mixed_c$m.$round.json 2> $O/mixed_c$m.$round.err
    python -c "import json; d=json.load(open('$O/mixed_c$m.$round.json')); print('concurrent=$m r$round', round(d['value']/1e6,2), d['roofline']['avg_launch_ms'], d['ms_per_step'])"
  done
done
