# multiplier-table codec: parity + exhaustive digests + bench
set -u
O=gpurun_out/r2c; mkdir -p $O
fatal() { rc=$1; if [ $rc -ge 124 ]; then echo "fatal rc=$rc ($2)"; exit $rc; fi; }
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -15 $O/pytest_gpu.log; fatal $rc pytest
[ $rc -ne 0 ] && exit 1
timeout -k 10 400 python bench.py --no-cpu-baseline > $O/bench.json 2> $O/bench.err; rc=$?; echo "bench rc=$rc"; fatal $rc bench
python3 -c "
import json; r=json.loads(open('$O/bench.json').read().strip().splitlines()[-1])
print('mnist64', r['value'], r['kernels'])
for k,v in r['extra'].items(): print(k, v['gib_s'], v['update_kernel_ms'], v['encode_kernel_ms'], v['update_kernel'])"
