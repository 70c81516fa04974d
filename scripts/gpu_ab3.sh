# A/B/C: ab/libfleetcodec_prev.so (A), fleet_amd/libfleetcodec.so (B), ab/libfleetcodec_c.so (C), same box
set -u
summ() { python3 -c "
import json,sys; r=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], 'mnist64', round(r['value'],1), round(r['kernels']['k_update_ms']*1e3,2), round(r['kernels']['k_encode_f32_ms']*1e3,2), end=' | ')
for k,v in r['extra'].items(): print(k, round(v['gib_s'],1), round(v['update_kernel_ms'],4), round(v['encode_kernel_ms'],4), end=' | ')
print()" $1 $2; }
for i in 1 2; do
  FLEET_CODEC_LIB=$PWD/ab/libfleetcodec_prev.so timeout -k 10 300 python bench.py --no-cpu-baseline --no-e2e > gpurun_out/ab_A$i.json 2>/dev/null || exit 1; summ gpurun_out/ab_A$i.json A
  timeout -k 10 300 python bench.py --no-cpu-baseline --no-e2e > gpurun_out/ab_B$i.json 2>/dev/null || exit 1; summ gpurun_out/ab_B$i.json B
  FLEET_CODEC_LIB=$PWD/ab/libfleetcodec_c.so timeout -k 10 300 python bench.py --no-cpu-baseline --no-e2e > gpurun_out/ab_C$i.json 2>/dev/null || exit 1; summ gpurun_out/ab_C$i.json C
done
