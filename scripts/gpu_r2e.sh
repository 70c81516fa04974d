# pipelined tile kernel phases (consumer priority, mulhi code step) + bench
set -u
O=gpurun_out/r2e; mkdir -p $O
timeout -k 10 120 ./scripts/ubench_tiled > $O/ubench_tiled.txt 2>&1; rc=$?; echo "ubench rc=$rc"; cat $O/ubench_tiled.txt; [ $rc -ge 124 ] && exit $rc
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -k "update or digest" > $O/pytest.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -3 $O/pytest.log; [ $rc -ge 124 ] && exit $rc
timeout -k 10 300 python bench.py --no-cpu-baseline --extras= > $O/bench.json 2> $O/bench.err; echo "bench rc=$?"; python3 -c "
import json; r=json.loads(open('$O/bench.json').read().strip().splitlines()[-1]); print('mnist64', r['value'], r['ms_per_step'], r['kernels'])"
