# byte-table tiles: narrow-tile width of the two-width grid (FLEET_TILE_MIX 16 / 32) on the CIFAR updates
set -u
one() { # $1 = label, $2 = workload, rest = env
  local lab=$1 w=$2; shift 2
  env "$@" timeout -k 10 300 python bench.py --workload $w --extras= --no-cpu-baseline --no-e2e --no-strong-block --steps 20 --warmup 3 > gpurun_out/abw.json 2>/dev/null || exit 1
  python3 -c "
import json; r=json.loads(open('gpurun_out/abw.json').read().strip().splitlines()[-1])
print('$lab', '$w', r['update_kernel'] if 'update_kernel' in r else '', 'update', round(r['kernels']['k_update_ms']*1e3,1), 'us  step', round(r['ms_per_step']*1e3,1))"
}
for rep in 1 2 3; do
  for w in cifar10_256 cifar100_1024; do
    one T16 $w FLEET_TILE_MIX=16
    one T32 $w FLEET_TILE_MIX=32
  done
done
