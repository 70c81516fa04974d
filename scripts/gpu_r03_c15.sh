# encode-wave priority in the fused steps (FLEET_FUSED_ENC_PRIO 0..3), alternating on one box
set -u
one() { # $1 = label, $2 = workload, rest = env
  local lab=$1 w=$2; shift 2
  env "$@" timeout -k 10 300 python bench.py --workload $w --extras= --no-cpu-baseline --no-e2e --no-strong-block --steps 20 --warmup 3 > gpurun_out/abw.json 2>/dev/null || exit 1
  python3 -c "
import json; r=json.loads(open('gpurun_out/abw.json').read().strip().splitlines()[-1])
print('$lab', '$w', 'update', round(r['kernels']['k_update_ms']*1e3,1), 'us  step', round(r['ms_per_step']*1e3,1), 'us  fused', round(r['pipelined']['kernel_ms']*1e3,1), 'us  sequential', round(r['sequential']['ms_per_step']*1e3,1))"
}
for rep in 1 2; do
  for w in synth1m_256 cifar10_256; do
    for p in 0 1 2 3; do one P$p $w FLEET_FUSED_ENC_PRIO=$p; done
  done
done
