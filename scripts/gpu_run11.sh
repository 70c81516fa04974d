set -u
mkdir -p gpurun_out
timeout -k 10 120 ./scripts/ubench_tiled > gpurun_out/ubench_tiled.log 2>&1 && cat gpurun_out/ubench_tiled.log &&
timeout -k 10 600 python -m pytest tests -m gpu -q -x > gpurun_out/pytest_gpu.log 2>&1; tail -3 gpurun_out/pytest_gpu.log
timeout -k 10 300 python bench.py --steps 20 --warmup 3 --cpu-budget 4 > gpurun_out/bench_r11.log 2>&1; tail -1 gpurun_out/bench_r11.log | python -c "
import json,sys; d=json.loads(sys.stdin.read()); print('value',round(d['value'],1),'ms',round(d['ms_per_step']*1e3,1),'us', d['kernels'], d['roofline']['frac'], d['end_to_end_host_buffers'])
print({k:(round(v['gib_s'],1), round(v['update_kernel_ms'],3), round(v['encode_kernel_ms'],3)) for k,v in d['extra'].items()})"
