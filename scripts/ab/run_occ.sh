#!/bin/bash
# Occupancy A/B (experiment): k_step with its SGPR budget cut so more workgroups fit per CU
# (gfx950 admits min(8, floor(800 / (ceil(sgpr/16)*16 + 16))) 256-lane blocks per CU).
#   base: product (105 SGPRs -> 6 / CU), s94 (94 -> 7 / CU), w8 (76 SGPRs, 64 VGPRs -> 8 / CU)
# quick parity of each experiment library first, then interleaved headline benches, then
# SQ occupancy counters of the headline for base and the best candidate.
set -euo pipefail
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
O=gpurun_out/${1:-occ}; mkdir -p $O
L=microrts-py_amd/gym_microrts/libmicrorts_amd.so
cp $L /tmp/lib_product.so
for v in s94 w8; do
  cp scripts/ab/lib$v.so $L
  timeout -k 10 400 python scripts/ab/quick_parity.py > $O/parity_$v.log 2>&1 && echo "parity ok $v" || { echo "parity FAILED $v"; tail -5 $O/parity_$v.log; }
done
for round in 1 2 3; do
  for v in base s94 w8; do
    cp scripts/ab/lib$v.so $L
    timeout -k 10 200 python bench.py --no-cpu-baseline --steps 150 > $O/head_$v.$round.json 2>/dev/null
    echo "$v $round head $(python -c "import json; d=json.load(open('$O/head_$v.$round.json')); print(d['value'], round(d['kernels']['step']['avg_ms']*1000,1), round(d['kernels']['sample']['avg_ms']*1000,1))")"
  done
done
B="bench.py --steps 40 --warmup 10 --no-cpu-baseline --no-kernel-events"
for v in base s94 w8; do
  cp scripts/ab/lib$v.so $L
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS GRBM_GUI_ACTIVE -f csv -d "$O/sq_$v/a" -o a -- python3 $B > /dev/null 2> "$O/sq_$v.a.err"
  timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS SQ_INSTS_SALU -f csv -d "$O/sq_$v/b" -o b -- python3 $B > /dev/null 2> "$O/sq_$v.b.err"
  python3 scripts/sq_summary.py "$O/sq_$v" "$O/sq_$v.json" "$B ($v)"
  rm -rf "$O/sq_$v"   # raw rocprof output: keeps gpurun_out under the 64 MiB copy-back limit
done
cp /tmp/lib_product.so $L
echo done > $O/DONE
