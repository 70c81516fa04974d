set -u
mkdir -p gpurun_out/r15
O=gpurun_out/r15
timeout -k 10 600 python -m pytest tests -m gpu -q -x > $O/pytest_gpu.log 2>&1; tail -2 $O/pytest_gpu.log
timeout -k 10 300 python bench.py --cpu-budget 4 > $O/bench.log 2>&1; echo "bench rc=$?"
tail -1 $O/bench.log | python -c "
import json,sys; d=json.loads(sys.stdin.read()); print('value',round(d['value'],1),'ms',round(d['ms_per_step']*1e3,1),'us', d['timing'], {k:round(v,4) for k,v in d['kernels'].items()}, d['roofline'], d['cpu_baseline']['value'], d['end_to_end_host_buffers'])
print({k:(round(v['gib_s'],1), v['update_kernel'], round(v['update_kernel_ms'],3), round(v['encode_kernel_ms'],3), round(v['ms_per_step'],3), round(v['eager_ms_per_step'],3)) for k,v in d['extra'].items()})"
