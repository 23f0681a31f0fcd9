#!/bin/bash
# k_sample_src groups-per-wave A/B: sampler parity tests per lib, then interleaved bench runs
# (headline + configs[1]) reporting the sampler's and the step kernel's HIP-event means.
set -euo pipefail
cd "${GRAFT_REPO_ROOT}"
O=gpurun_out/$1; mkdir -p $O
L=microrts-py_amd/gym_microrts/libmicrorts_amd.so
cp $L /tmp/lib_product.so
for v in $2; do
  cp scripts/ab/lib$v.so $L
  if ! timeout -k 10 300 python -m pytest tests/test_gpu_parity.py tests/test_gpu_shard.py -m gpu -q -k "sampler" > $O/parity_$v.txt 2>&1; then
    echo "PARITY FAIL $v"; tail -15 $O/parity_$v.txt; cp /tmp/lib_product.so $L; exit 1
  fi
  case $v in *i) timeout -k 10 400 python scripts/ab/quick_parity.py > $O/qparity_$v.txt 2>&1 || { echo "ENGINE PARITY FAIL $v"; tail -5 $O/qparity_$v.txt; cp /tmp/lib_product.so $L; exit 1; };; esac
  echo "parity ok $v: $(tail -1 $O/parity_$v.txt)"
done
for round in $(seq 1 ${3:-2}); do
  for v in $2; do
    cp scripts/ab/lib$v.so $L
    timeout -k 10 200 python bench.py --no-cpu-baseline --steps 150 > $O/head_$v.$round.json 2>/dev/null
    timeout -k 10 200 python bench.py --workload coac --envs-per-gpu 1024 --no-cpu-baseline --steps 300 > $O/coac_$v.$round.json 2>/dev/null
    python - $O/head_$v.$round.json $O/coac_$v.$round.json $v $round <<'PY'
import json, sys
out = []
for f in sys.argv[1:3]:
    d = json.load(open(f)); k = d["kernels"]
    out.append(f"{d['value']/1e6:.2f}M sample {k['sample']['avg_ms']*1e3:.1f} step {k['step']['avg_ms']*1e3:.1f}")
print(sys.argv[3], sys.argv[4], "head", out[0], "| coac", out[1])
PY
  done
done
cp /tmp/lib_product.so $L
