#!/bin/bash
# One gpurun call: the headline and configs[1] as medians of 3 seeds, every secondary
# BASELINE.json config, and the reference's numpy contract (PCIe-inclusive).
#   /usr/local/graft/bin/gpurun --timeout 1200 -- bash scripts/gpu_configs.sh TAG
set -euo pipefail
TAG=${1:-run}
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/$TAG
mkdir -p "$O"
timeout -k 10 400 python bench.py --seeds 3 --no-cpu-baseline > "$O/selfplay_3seeds.json" 2> "$O/selfplay.err"
timeout -k 10 300 python bench.py --workload coac --envs-per-gpu 1024 --seeds 3 --no-cpu-baseline > "$O/coac_1024_3seeds.json" 2> "$O/coac.err"
for spec in "passive 8192" "coac 8192" "workerrush 8192" "partial_obs 4096" "partial_obs 8192" "mixed 8192" "8x8 8192" "24x24 8192"; do
  set -- $spec
  timeout -k 10 300 python bench.py --workload "$1" --envs-per-gpu "$2" --steps 200 --warmup 30 --no-cpu-baseline > "$O/$1_$2.json" 2> "$O/$1_$2.err"
done
timeout -k 10 300 python bench.py --api numpy --steps 30 --warmup 5 --no-cpu-baseline > "$O/numpy_8192.json" 2> "$O/numpy.err"
python - "$O" <<'PY'
import glob, json, os, sys
for f in sorted(glob.glob(os.path.join(sys.argv[1], "*.json"))):
    d = json.loads(open(f).read().strip().splitlines()[-1])
    r = d.get("roofline") or {}
    print(f"{os.path.basename(f):28s} {d['value']/1e6:8.3f} M  frac {r.get('frac')}  step {r.get('avg_launch_ms')}")
PY
