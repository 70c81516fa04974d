# cifar10_256 aggregation kernel choices (same box)
set -u
run() { env "$@" timeout -k 10 300 python bench.py --workload cifar10_256 --extras= --no-cpu-baseline --no-e2e --steps 8 --warmup 2 > gpurun_out/cs.json 2>/dev/null || exit 1
  python3 -c "import json; r=json.loads(open('gpurun_out/cs.json').read().strip().splitlines()[-1]); print('$*', r['roofline']['kernel'], round(r['kernels']['k_update_ms']*1e3,1), 'us')"; }
run A=1
run FLEET_UPDATE_MODE=stream FLEET_UPDATE_K=1
run FLEET_TILE_G=32
run FLEET_TILE_G=16 FLEET_UPDATE_PIPE=0
run FLEET_TILE_G=16
run FLEET_TILE_G=64
