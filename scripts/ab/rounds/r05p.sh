#!/bin/bash
# Round 5: instruction-cache counters of configs[1]'s fused step kernel (is the latency-
# bound bot wave fetch-bound?) and of the headline's step kernel for comparison
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out/r05p; mkdir -p $O
for W in coac selfplay; do
  if [ $W = selfplay ]; then B="bench.py --steps 40 --warmup 10 --no-cpu-baseline --no-kernel-events"
  else B="bench.py --workload coac --envs-per-gpu 1024 --steps 100 --warmup 10 --no-cpu-baseline --no-kernel-events"; fi
  timeout -s KILL 300 rocprofv3 --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQC_ICACHE_REQ SQ_IFETCH SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_SALU -f csv -d "$O/ic_$W/a" -o a -- python3 $B > /dev/null 2> "$O/ic_$W.a.err"
  python3 scripts/sq_summary.py "$O/ic_$W" "$O/ic_$W.json" "$B"
  rm -rf "$O/ic_$W"
  python3 - "$O/ic_$W.json" <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
for k, v in d["kernels"].items():
    c = v["counters"]
    if "SQC_ICACHE_REQ" in c and c["SQC_ICACHE_REQ"]:
        print(k[:40], {a: round(b) for a, b in c.items()}, "miss/req", round(c["SQC_ICACHE_MISSES"] / c["SQC_ICACHE_REQ"], 4))
PY
done
