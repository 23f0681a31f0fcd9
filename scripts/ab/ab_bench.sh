#!/bin/bash
# Same-box interleaved A/B of library builds: for each round, each variant .so is
# copied over the product library path and the bench command is run; the product
# build is restored at the end.  One JSON line per (round, variant) in $O.
#   bash scripts/ab/ab_bench.sh OUTDIR ROUNDS "bench args" variant1.so variant2.so ...
# ("cur" as a variant = the working tree's build)
set -euo pipefail
O=$1; R=$2; ARGS=$3; shift 3
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
L=microrts-py_amd/gym_microrts/libmicrorts_amd.so
mkdir -p "$O"
cp "$L" "$O/.cur.so"
trap 'cp "$O/.cur.so" "$L"; rm -f "$O/.cur.so"' EXIT
for r in $(seq 1 "$R"); do
  for v in "$@"; do
    n=$(basename "$v" .so)
    if [ "$v" = cur ]; then cp "$O/.cur.so" "$L"; else cp "$v" "$L"; fi
    timeout -k 10 300 python bench.py $ARGS --no-cpu-baseline > "$O/${n}_r$r.json" 2> "$O/${n}_r$r.err"
    python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d.get('roofline') or {}; print(sys.argv[2], sys.argv[3], round(d['value']/1e6,3), 'M', r.get('avg_launch_ms'), r.get('frac'))" "$O/${n}_r$r.json" "$n" "$r"
  done
done
