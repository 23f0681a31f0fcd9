#!/bin/bash
# Round 5: configs[4]'s stand-in policy in one launch over the three size buckets
# (mrts_sample_actions_src_group) vs one mrts_sample_actions_src launch per bucket; same
# library, same actions; interleaved rounds on one box.
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r05r; mkdir -p $O
timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k "sampler" > $O/pytest_sampler.log 2>&1
tail -1 $O/pytest_sampler.log
for r in 1 2 3; do
  for g in 0 1; do
    timeout -k 10 300 python bench.py --workload mixed --envs-per-gpu 8192 --steps 200 --warmup 30 --no-cpu-baseline --sampler-group $g > $O/mixed_g${g}_r$r.json 2> $O/mixed_g${g}_r$r.err
    python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('group', sys.argv[2], 'round', sys.argv[3], round(d['value']/1e6,3), 'M', d['ms_per_step'], d['roofline']['avg_launch_ms'], d['window'].get('sampler_launches_per_step'))" $O/mixed_g${g}_r$r.json $g $r
  done
done
