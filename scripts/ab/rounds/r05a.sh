#!/bin/bash
# Round 5, first GPU call: the new / changed GPU tests (4-rank self-launch, configs[4]
# at the bench's size, trained-policy lock-step, produce budget boundary, checkpoint
# fingerprint, sampler parity), then the write-first sampler A/B (prev = HEAD before it).
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r05a; mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread -m gpu \
  tests/test_gpu_produce_budget.py tests/test_gpu_checkpoint.py tests/test_gpu_shard.py tests/test_gpu_policy.py \
  "tests/test_gpu_fullsize.py::test_fullsize_mixed_buckets_bench_split_8192" -k "not two_shards" \
  > $O/pytest_new.txt 2>&1 || { tail -40 $O/pytest_new.txt; exit 1; }
tail -2 $O/pytest_new.txt
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "sampler" > $O/pytest_sampler.txt 2>&1 || { tail -40 $O/pytest_sampler.txt; exit 1; }
tail -1 $O/pytest_sampler.txt
bash scripts/ab/ab_bench.sh $O/selfplay 3 "--steps 200 --warmup 30" scripts/ab/libs/prev.so cur
