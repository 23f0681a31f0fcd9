#!/bin/bash
set -euo pipefail
cd "${GRAFT_REPO_ROOT}"
O=gpurun_out/$1; mkdir -p $O
for r in 1 2 3; do
  for v in old new; do
    if [ $v = old ]; then S=scripts/ab/${OLD:-shm_old.py}; else S=bench.py; fi
    timeout -k 10 300 python $S --api ${API:-sharedmem} --steps 30 --warmup 5 --no-cpu-baseline > $O/shm_$v.$r.json 2> $O/shm_$v.$r.err
    python -c "import json; d=json.load(open('$O/shm_$v.$r.json')); print('$v r$r', round(d['value']/1e3,1), 'k', d['ms_per_step'])"
  done
done
