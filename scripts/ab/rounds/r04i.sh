#!/bin/bash
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r04i; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 280 --timeout-method thread tests/test_gpu_bots.py tests/test_gpu_parity.py tests/test_gpu_render.py -k "lockstep or render or other_maps" > $O/pytest.txt 2>&1 || { tail -30 $O/pytest.txt; exit 1; }
tail -1 $O/pytest.txt
for L in stamps stamps_pad16; do
  for spec in "coac 1024" "selfplay 8192"; do
    set -- $spec
    timeout -k 10 240 python -u scripts/stamps_run.py --lib scripts/ab/libs/$L.so --workload $1 --envs-per-gpu $2 --steps 20 --json $O/st_${L}_$1_$2.json > $O/st_${L}_$1_$2.txt 2>&1
  done
done
bash scripts/ab/ab_bench.sh $O/selfplay 2 "--steps 200 --warmup 30" cur scripts/ab/libs/pad16.so
bash scripts/ab/ab_bench.sh $O/coac1024 2 "--workload coac --envs-per-gpu 1024 --steps 300 --warmup 30" cur scripts/ab/libs/pad16.so
for spec in "coac 1024"; do
  set -- $spec
  timeout -k 10 240 python -u scripts/stamps_run.py --lib scripts/ab/libs/stamps_deferaa.so --workload $1 --envs-per-gpu $2 --steps 20 --json $O/st_stamps_deferaa_$1_$2.json > $O/st_stamps_deferaa_$1_$2.txt 2>&1
done
bash scripts/ab/ab_bench.sh $O/coac1024b 2 "--workload coac --envs-per-gpu 1024 --steps 300 --warmup 30" cur scripts/ab/libs/deferaa.so
