# encode rows-per-block sweep (FLEET_ENCODE_RPB) on synth1m_256: k_encode_f32 time per setting
set -u
for R in ${RPBS:-2 4 6 8 12 16 24 32}; do
  FLEET_ENCODE_RPB=$R timeout -k 10 300 python bench.py --workload ${WL:-synth1m_256} --extras= --no-cpu-baseline --no-e2e --no-strong-block --steps 20 --warmup 3 > gpurun_out/rpb.json 2>/dev/null || exit 1
  python3 -c "
import json; r=json.loads(open('gpurun_out/rpb.json').read().strip().splitlines()[-1])
print('rpb $R encode', round(r['kernels']['k_encode_f32_ms']*1e3,1), 'us  step', round(r['ms_per_step']*1e3,1), 'sequential', round(r['sequential']['ms_per_step']*1e3,1), 'fused', round(r['roofline']['kernel_ms']*1e3,1))"
done
