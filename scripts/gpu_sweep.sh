# kernel choices on one workload (W, default mnist64; same box); each configuration run twice
set -u
run() { env "$@" timeout -k 10 300 python bench.py --workload ${W:-mnist64} --extras= --no-cpu-baseline --no-e2e --steps 50 --warmup 5 > gpurun_out/ms.json 2>/dev/null || exit 1
  python3 -c "import json; r=json.loads(open('gpurun_out/ms.json').read().strip().splitlines()[-1]); print('$*', r['roofline']['kernel'], round(r['kernels']['k_update_ms']*1e3,2), 'us', round(r['kernels']['k_encode_f32_ms']*1e3,2), 'us enc', round(r['ms_per_step']*1e3,2), 'us/step')"; }
# SWEEP: configurations separated by ';' (each a list of VAR=value)
SWEEP=${SWEEP:-"A=1;FLEET_TILE_G=8;FLEET_TILE_G=8 FLEET_PIPE_WAVES=4;FLEET_TILE_G=8 FLEET_PIPE_WAVES=8;FLEET_TILE_G=16 FLEET_PIPE_WAVES=8"}
IFS=';' read -ra CFGS <<< "$SWEEP"
for rep in 1 2; do
  for cfg in "${CFGS[@]}"; do
    read -ra kv <<< "$cfg"
    run "${kv[@]}"
  done
done
