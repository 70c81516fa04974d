set -u
O=gpurun_out/r2j; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -k "update or digest or model" > $O/pytest.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -2 $O/pytest.log; [ $rc -ne 0 ] && exit 1
timeout -k 10 300 python bench.py --no-cpu-baseline --no-e2e > $O/bench.json 2> $O/bench.err; echo "bench rc=$?"; python3 -c "
import json; r=json.loads(open('$O/bench.json').read().strip().splitlines()[-1]); print('mnist64', r['value'], r['ms_per_step'], r['kernels']['k_update_ms'], r['kernels']['k_encode_f32_ms'])
for k,v in r['extra'].items(): print(k, v['gib_s'], v['ms_per_step'], v['update_kernel_ms'], v['encode_kernel_ms'])"
