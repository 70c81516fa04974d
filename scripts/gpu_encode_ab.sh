# client-encode A/B on one box: FLEET_ENCODE_D16 (byte-table vs VarEntry digit counts) x rows per block,
# alternating, on synth1m_256 (k_encode_f32 alone, sequential step, the fused pipelined step)
set -u
for rep in 1 2; do
for D in 0 1; do for R in ${RPBS:-6 12}; do
  FLEET_ENCODE_D16=$D FLEET_ENCODE_RPB=$R timeout -k 10 300 python bench.py --workload ${WL:-synth1m_256} --extras= --no-cpu-baseline --no-e2e --no-strong-block --steps 20 --warmup 3 > gpurun_out/eab.json 2>/dev/null || exit 1
  python3 -c "
import json; r=json.loads(open('gpurun_out/eab.json').read().strip().splitlines()[-1])
print('d16 $D rpb $R encode', round(r['kernels']['k_encode_f32_ms']*1e3,1), 'us  step', round(r['ms_per_step']*1e3,1), 'sequential', round(r['sequential']['ms_per_step']*1e3,1), 'fused', round(r['roofline']['kernel_ms']*1e3,1))"
done; done; done
