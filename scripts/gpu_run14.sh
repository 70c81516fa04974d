set -u
mkdir -p gpurun_out/r14
O=gpurun_out/r14
timeout -k 10 120 ./scripts/ubench_tiled > $O/ubench_tiled.log 2>&1 && head -3 $O/ubench_tiled.log &&
for G in 0 1; do
timeout -k 10 300 python bench.py --steps 50 --warmup 5 --no-cpu-baseline --graph $G > $O/bench_g$G.log 2>&1; echo "bench g$G rc=$?"
tail -1 $O/bench_g$G.log | python -c "
import json,sys; d=json.loads(sys.stdin.read()); print('value',round(d['value'],1),'ms',round(d['ms_per_step']*1e3,1),'us', {k:round(v,4) for k,v in d['kernels'].items()}, 'frac', round(d['roofline']['frac'],4), d['end_to_end_host_buffers'])
print({k:(round(v['gib_s'],1), round(v['update_kernel_ms'],3), round(v['encode_kernel_ms'],3), round(v['eager_ms_per_step'],3)) for k,v in d['extra'].items()})"
done
