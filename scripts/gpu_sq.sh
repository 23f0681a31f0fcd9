#!/bin/bash
# SQ counters of the step kernel for the headline and configs[1] bench commands (two passes each:
# rocprofv3 does not split counters over passes; <= 8 SQ_ + 1 GRBM_ per pass)
#   /usr/local/graft/bin/gpurun --timeout 900 -- bash scripts/gpu_sq.sh TAG
set -euo pipefail
TAG=${1:-sq}
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/$TAG
mkdir -p "$O"
for W in selfplay coac; do
  if [ $W = selfplay ]; then B="bench.py --steps 40 --warmup 10 --no-cpu-baseline --no-kernel-events"
  else B="bench.py --workload coac --envs-per-gpu 1024 --steps 100 --warmup 10 --no-cpu-baseline --no-kernel-events"; fi
  timeout -s KILL 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS GRBM_GUI_ACTIVE -f csv -d "$O/sq_$W/a" -o a -- python3 $B > /dev/null 2> "$O/sq_$W.a.err"
  timeout -s KILL 300 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS SQ_INSTS_SALU -f csv -d "$O/sq_$W/b" -o b -- python3 $B > /dev/null 2> "$O/sq_$W.b.err"
  python3 scripts/sq_summary.py "$O/sq_$W" "$O/sq_$W.json" "$B"
  rm -rf "$O/sq_$W"   # raw rocprof output: keeps gpurun_out under the 64 MiB copy-back limit
done
echo done > "$O/DONE"
