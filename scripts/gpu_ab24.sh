set -euo pipefail
O=gpurun_out/r01z8; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_bots.py -k "other_maps or adversarial" -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for f in 0 1; do timeout -k 10 300 python bench.py --workload mixed --envs-per-gpu 8192 --steps 200 --warmup 30 --no-cpu-baseline --bot-fusion $f > $O/mixed_f$f.json 2> $O/mixed_f$f.err; done
for f in $O/*.json; do python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[1], round(d['value']/1e6,2))" $f; done
