# fused-step A/B on one box, alternating: environment settings of k_update_encode (default: the plain
# stream grid inside the fused kernel vs the SIMD-balanced one)
set -u
for rep in 1 2 3; do
for V in ${VARIANTS:-FLEET_FUSED_PLAIN=0 FLEET_FUSED_PLAIN=1}; do  # 0: SIMD-balanced grid, 1: plain (default)
  env $V timeout -k 10 300 python bench.py --workload ${WL:-synth1m_256} --extras= --no-cpu-baseline --no-e2e --no-strong-block --steps 20 --warmup 3 > gpurun_out/fab.json 2>/dev/null || exit 1
  python3 -c "
import json; r=json.loads(open('gpurun_out/fab.json').read().strip().splitlines()[-1])
print('$V step', round(r['ms_per_step']*1e3,1), 'fused', round(r['roofline']['kernel_ms']*1e3,1), 'update alone', round(r['kernels']['k_update_ms']*1e3,1))"
done; done
