# host-buffer update (fleet_update) staging sweep: FLEET_STAGE_THREADS x FLEET_STAGE_PIECES on the e2e workloads
set -u
O=gpurun_out/e2e_sweep; mkdir -p $O
for cfg in ${CFGS:-"T=1 P=1" "T=2 P=1" "T=2 P=3" "T=4 P=3" "T=8 P=3" "T=8 P=9" "T=8 P=16" "T=16 P=9"}; do
  eval $cfg
  FLEET_STAGE_THREADS=$T FLEET_STAGE_PIECES=$P timeout -k 10 300 python bench.py --workload mnist64 --extras= --no-cpu-baseline --no-strong-block --steps 3 --e2e ${E2E:-mnist64,cifar10_256} > $O/b.json 2>/dev/null || exit 1
  python3 -c "
import json; d=json.loads(open('$O/b.json').read().strip().splitlines()[-1])
print('$cfg', ' '.join(f\"{k}: {v['ms']:.3f} ms x{v['x_floor']:.2f}\" for k,v in d['end_to_end_host_buffers'].items()))"
done
