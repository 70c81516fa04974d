set -u
for i in 1 2 3; do
timeout -k 10 300 python bench.py --no-cpu-baseline --no-e2e > gpurun_out/r2l_$i.json 2>/dev/null; python3 -c "
import json; r=json.loads(open('gpurun_out/r2l_$i.json').read().strip().splitlines()[-1]); print('mnist64', round(r['value'],1), round(r['kernels']['k_update_ms']*1e3,2), round(r['kernels']['k_encode_f32_ms']*1e3,2), end=' | ')
for k,v in r['extra'].items(): print(k, round(v['gib_s'],1), round(v['update_kernel_ms'],4), round(v['encode_kernel_ms'],4), end=' | ')
print()"
done
