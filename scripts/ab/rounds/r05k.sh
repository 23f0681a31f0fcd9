#!/bin/bash
# Round 5: (1) the sampler walking rows newest-written first; (2) the upper bound of a
# tail split (timing only, wrong outputs): the last X games' second env's mask rows are
# written by X extra helper workgroups (zeros after a 12 us sleep standing in for the
# logic), the primaries write only the first env's -- what halving the tail games'
# streams could save.
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
O=gpurun_out/r05k; mkdir -p $O
bash scripts/ab/ab_bench.sh $O/selfplay 3 "--steps 200 --warmup 30" cur scripts/ab/libs/sampler_rev.so scripts/ab/libs/tail512.so scripts/ab/libs/tail1024.so
