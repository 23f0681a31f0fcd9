#!/bin/bash
# Round 5: trained-policy lock-step on 8x8 / 24x24 / 16x16 with every device bot kind
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r05l; mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread -m gpu tests/test_gpu_policy.py > $O/pytest_policy.txt 2>&1 || { tail -40 $O/pytest_policy.txt; exit 1; }
grep -E "PASS|FAIL|passed|failed" $O/pytest_policy.txt | tail -6
