# encode inside the tiles (FLEET_FUSED_TILE_INLINE): fused-step tests, then 0 / 1 on the CIFAR workloads
set -u
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu \
  tests/test_gpu_fused_step.py tests/test_gpu_full_size.py > gpurun_out/c16_tests.log 2>&1 || { tail -30 gpurun_out/c16_tests.log; exit 1; }
tail -1 gpurun_out/c16_tests.log
one() { # $1 = label, $2 = workload, rest = env
  local lab=$1 w=$2; shift 2
  env "$@" timeout -k 10 300 python bench.py --workload $w --extras= --no-cpu-baseline --no-e2e --no-strong-block --steps 20 --warmup 3 > gpurun_out/abw.json 2>/dev/null || exit 1
  python3 -c "
import json; r=json.loads(open('gpurun_out/abw.json').read().strip().splitlines()[-1])
print('$lab', '$w', r['pipelined']['kernel'], 'update', round(r['kernels']['k_update_ms']*1e3,1), 'us  step', round(r['ms_per_step']*1e3,1), 'us  fused', round(r['pipelined']['kernel_ms']*1e3,1), 'us  sequential', round(r['sequential']['ms_per_step']*1e3,1))"
}
for rep in 1 2; do
  for w in cifar10_256 cifar100_1024; do
    one I0 $w FLEET_FUSED_TILE_INLINE=0
    one I1 $w FLEET_FUSED_TILE_INLINE=1
  done
done
