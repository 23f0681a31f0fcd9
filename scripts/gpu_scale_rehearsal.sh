#!/bin/bash
# Rehearsal of the driver's SCALE invocation on a 1-GPU box: N ranks of the default
# bench (8192 envs each, gloo timing group) all on the box's one GPU -- the
# launcher, rendezvous, per-rank gather and line are exercised end to end; the numbers
# are N ranks sharing one GPU, not a scaling curve.
#   /usr/local/graft/bin/gpurun --timeout 900 -- bash scripts/gpu_scale_rehearsal.sh TAG
set -euo pipefail
TAG=${1:-scale_rehearsal}
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/$TAG
mkdir -p "$O"
PORT=$(python -c "import socket; s=socket.socket(); s.bind(('127.0.0.1',0)); print(s.getsockname()[1])")
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port "$PORT" \
  bench.py --gpus 8 --steps 50 --warmup 10 > "$O/torchrun_8.json" 2> "$O/torchrun_8.err"
timeout -k 10 600 python bench.py --gpus 4 --steps 50 --warmup 10 > "$O/self_4.json" 2> "$O/self_4.err"
python - "$O" <<'PY'
import glob, json, os, sys
for f in sorted(glob.glob(os.path.join(sys.argv[1], "*.json"))):
    d = json.loads([l for l in open(f) if l.startswith("{")][-1])
    w = d["window"]
    print(os.path.basename(f), d["n_gpus"], d["process_group"], round(d["value"] / 1e6, 3), "M",
          [round(p["env_steps_per_s"] / 1e6, 3) for p in w["per_rank"]], w.get("per_rank_spread"))
PY
