#!/bin/bash
# configs[4] launch grouping: the mixed / step-group parity tests, then the mixed bench
# under each mrts_step_group policy, interleaved rounds on one box.
#   /usr/local/graft/bin/gpurun --timeout 900 -- bash scripts/gpu_group_ab.sh TAG [ROUNDS]
set -euo pipefail
TAG=${1:-group}
ROUNDS=${2:-2}
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/$TAG
mkdir -p "$O"
timeout -k 10 600 python -u -m pytest tests/test_gpu_bots.py -m gpu -x -v --timeout 300 --timeout-method thread \
  -k "mixed or step_group" > "$O/pytest.log" 2>&1 || { echo "pytest failed"; tail -40 "$O/pytest.log"; exit 1; }
tail -2 "$O/pytest.log"
for r in $(seq 1 "$ROUNDS"); do
  for pol in none 0 1 5 2 6; do
    timeout -k 10 300 python bench.py --workload mixed --steps 200 --warmup 30 --group-policy "$pol" > "$O/mixed_${pol}_r$r.json" 2> "$O/mixed_${pol}_r$r.err"
    python - "$O/mixed_${pol}_r$r.json" "$pol" "$r" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
w = d["config"]; rf = d["roofline"]; s = d.get("window", {})
print(f"policy {sys.argv[2]:>4} round {sys.argv[3]}: {d['value']/1e6:.2f} M env-steps/s, step launches {rf['avg_launch_ms']*1e3:.1f} us, frac {rf['frac']:.3f}")
PY
  done
done
