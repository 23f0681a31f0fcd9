#!/bin/bash
# The product build in the tree (phase-B index math, fewer barriers, one bot_game call site,
# one copy of each bot routine: fused k_step 1 MB -> 166 KB of code, k_bot 468 -> 98 KB):
# the whole -m gpu suite, then interleaved headline / configs[1] benches of new (e565b84's
# kernels) vs head (this build), then instruction-cache counters of both on configs[1].
set -euo pipefail
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
O=gpurun_out/${1:-cs}; mkdir -p $O
L=microrts-py_amd/gym_microrts/libmicrorts_amd.so
cp $L /tmp/lib_product.so
restore() { cp /tmp/lib_product.so $L; }
trap restore EXIT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > $O/pytest_gpu.log 2>&1 \
  || { echo "pytest failed"; tail -40 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
for round in 1 2 3; do
  for v in new head; do
    cp scripts/ab/lib$v.so $L
    timeout -k 10 200 python bench.py --no-cpu-baseline --steps 150 > $O/head_$v.$round.json 2>/dev/null
    timeout -k 10 200 python bench.py --no-cpu-baseline --workload coac --envs-per-gpu 1024 --steps 300 > $O/coac_$v.$round.json 2>/dev/null
    echo "$v $round head $(python -c "import json; d=json.load(open('$O/head_$v.$round.json')); print(d['value'], round(d['kernels']['step']['avg_ms']*1000,1), round(d['kernels']['sample']['avg_ms']*1000,1))") coac $(python -c "import json; d=json.load(open('$O/coac_$v.$round.json')); print(d['value'], round(d['kernels']['step']['avg_ms']*1000,1), round(d['kernels']['sample']['avg_ms']*1000,1))")"
  done
done
B="bench.py --workload coac --envs-per-gpu 1024 --steps 100 --warmup 10 --no-cpu-baseline --no-kernel-events"
for v in new head; do
  cp scripts/ab/lib$v.so $L
  timeout -s KILL 120 rocprofv3 --pmc SQC_ICACHE_REQ SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE -f csv -d "$O/ic_$v/a" -o a -- python3 $B > /dev/null 2> "$O/ic_$v.a.err" || echo "pass a failed ($v): $(tail -2 $O/ic_$v.a.err)"
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_IFETCH SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS -f csv -d "$O/ic_$v/b" -o b -- python3 $B > /dev/null 2> "$O/ic_$v.b.err" || echo "pass b failed ($v): $(tail -2 $O/ic_$v.b.err)"
  python3 scripts/sq_summary.py "$O/ic_$v" "$O/ic_$v.json" "$B ($v)" > /dev/null
  python3 - "$O/ic_$v.json" "$v" <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
for k, v in d["kernels"].items():
    if k.startswith("k_step"):
        print(sys.argv[2], k, v["launches"], {a: round(b) for a, b in v["counters"].items()})
PY
  rm -rf "$O/ic_$v"
done
echo done > $O/DONE
