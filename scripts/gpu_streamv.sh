# value-per-lane stream kernel: parity, then same-box timing against k_update<1>
set -u
O=gpurun_out/sv; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "update" > $O/t.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -2 $O/t.log; [ $rc -ne 0 ] && exit 1
for i in 1 2; do for MODE in stream streamv; do
  FLEET_UPDATE_MODE=$MODE timeout -k 10 300 python bench.py --workload synth1m_256 --extras= --no-cpu-baseline --no-e2e --steps 8 --warmup 2 > $O/b.json 2>/dev/null || exit 1
  python3 -c "import json; r=json.loads(open('$O/b.json').read().strip().splitlines()[-1]); print('$MODE', r['roofline']['kernel'], round(r['kernels']['k_update_ms']*1e3,1), 'us', round(r['value'],1))"
done; done
