#!/bin/bash
# Instruction-cache counters of the step kernels: the bot-fused k_step carries the whole
# device bot inline (~1 MB of code), the headline kernel ~65 KB.  One pass per counter group.
#   /usr/local/graft/bin/gpurun --timeout 600 -- bash scripts/gpu_icache.sh TAG
set -uo pipefail
TAG=${1:-icache}
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/$TAG
mkdir -p "$O"
for W in coac selfplay; do
  if [ $W = selfplay ]; then B="bench.py --steps 40 --warmup 10 --no-cpu-baseline --no-kernel-events"
  else B="bench.py --workload coac --envs-per-gpu 1024 --steps 100 --warmup 10 --no-cpu-baseline --no-kernel-events"; fi
  timeout -s KILL 120 rocprofv3 --pmc SQC_ICACHE_REQ SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE -f csv -d "$O/ic_$W/a" -o a -- python3 $B > /dev/null 2> "$O/ic_$W.a.err" || echo "pass a failed ($W): $(tail -2 $O/ic_$W.a.err)"
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_IFETCH SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS -f csv -d "$O/ic_$W/b" -o b -- python3 $B > /dev/null 2> "$O/ic_$W.b.err" || echo "pass b failed ($W): $(tail -2 $O/ic_$W.b.err)"
  python3 scripts/sq_summary.py "$O/ic_$W" "$O/ic_$W.json" "$B"
  python3 - "$O/ic_$W.json" <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
for k, v in d["kernels"].items():
    if k.startswith("k_step") or k.startswith("k_bot") or k.startswith("k_sample"):
        print(k, v["launches"], {a: round(b) for a, b in v["counters"].items()})
PY
  rm -rf "$O/ic_$W"
done
echo done > "$O/DONE"
