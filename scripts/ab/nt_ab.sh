#!/bin/bash
# 512-lane step for maps > 256 cells: parity (parity + bot suites) on the new lib, then
# interleaved benches of the mixed config and 24x24 selfplay per lib.
set -euo pipefail
cd "${GRAFT_REPO_ROOT}"
O=gpurun_out/$1; mkdir -p $O
L=microrts-py_amd/gym_microrts/libmicrorts_amd.so
cp $L /tmp/lib_product.so
cp scripts/ab/lib$3.so $L
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_bots.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/parity_$3.txt 2>&1 \
  || { echo "PARITY FAIL"; tail -30 $O/parity_$3.txt; cp /tmp/lib_product.so $L; exit 1; }
echo "parity $3: $(tail -1 $O/parity_$3.txt)"
for round in 1 2; do
  for v in $2; do
    cp scripts/ab/lib$v.so $L
    timeout -k 10 300 python bench.py --workload mixed --no-cpu-baseline --steps 200 --warmup 30 > $O/mixed_$v.$round.json 2>/dev/null
    timeout -k 10 300 python bench.py --workload 24x24 --no-cpu-baseline --steps 100 --warmup 20 > $O/s24_$v.$round.json 2>/dev/null
    python - $O/mixed_$v.$round.json $O/s24_$v.$round.json $v $round <<'PY'
import json, sys
m = json.load(open(sys.argv[1])); s = json.load(open(sys.argv[2]))
print(sys.argv[3], sys.argv[4], f"mixed {m['value']/1e6:.2f}M step {m['roofline']['avg_launch_ms']*1e3:.1f}us frac {m['roofline']['frac']:.3f}",
      f"| 24x24 {s['value']/1e6:.2f}M step {s['kernels']['step']['avg_ms']*1e3:.1f}us frac {s['roofline']['frac']:.3f}")
PY
  done
done
cp /tmp/lib_product.so $L
