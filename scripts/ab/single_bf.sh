#!/bin/bash
set -euo pipefail
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out/$1
timeout -k 10 600 python -u scripts/ab/single_botsfirst.py | tee gpurun_out/$1/out.txt
