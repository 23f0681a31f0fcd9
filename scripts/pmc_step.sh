#!/bin/bash
# SQ counters of the step / masks / sample kernels (one pass each set).
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${1:-pmcstep}
mkdir -p "$O"
B="bench.py --steps 30 --warmup 10 --no-cpu-baseline --no-kernel-events"
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU -f csv -d "$O/a" -o a -- python3 $B > /dev/null 2> "$O/a.err"
timeout -k 10 300 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -f csv -d "$O/b" -o b -- python3 $B > /dev/null 2> "$O/b.err"
echo ok
