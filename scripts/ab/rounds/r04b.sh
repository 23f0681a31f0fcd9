#!/bin/bash
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r04b; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 280 --timeout-method thread tests/test_gpu_bots.py tests/test_gpu_fullsize.py tests/test_wall1_map.py tests/test_gpu_parity.py -k "partial or PO or wall1 or lockstep" > $O/pytest.txt 2>&1 || { tail -30 $O/pytest.txt; exit 1; }
tail -2 $O/pytest.txt
bash scripts/ab/ab_bench.sh $O/po 2 "--workload partial_obs --envs-per-gpu 4096 --steps 200 --warmup 30" scripts/ab/libs/head.so cur
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_mixed -o mixed -- python bench.py --workload mixed --steps 100 --warmup 10 --no-cpu-baseline > $O/mixed.json 2> $O/mixed.err
