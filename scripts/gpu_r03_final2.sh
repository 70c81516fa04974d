# round-3 check after the tile/Kardam changes: full GPU suite + smoke + default bench (gpu_final.sh),
# then the N=2 same-device rehearsal of bench.py's self-spawned ranks (gloo)
set -u
bash scripts/gpu_final.sh || exit 1
FLEET_BENCH_SAME_DEVICE=1 FLEET_BENCH_BACKEND=gloo timeout -k 10 400 python bench.py --gpus 2 --steps 3 --warmup 1 > gpurun_out/final/bench_n2_rehearsal.json 2> gpurun_out/final/bench_n2_rehearsal.err; echo "n2 rc=$?"
tail -c 400 gpurun_out/final/bench_n2_rehearsal.json
