# after the tile-width rule and the overlapped strong gather: full GPU suite + smoke + default bench,
# the N=2 same-device rehearsal (gloo) of the self-spawned ranks, the strong-scaling windows
set -u
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
bash scripts/gpu_final.sh || exit 1
FLEET_BENCH_SAME_DEVICE=1 FLEET_BENCH_BACKEND=gloo timeout -k 10 400 python bench.py --gpus 2 --steps 4 --warmup 1 > gpurun_out/final/bench_n2_rehearsal.json 2> gpurun_out/final/bench_n2_rehearsal.err; echo "n2 rc=$?"
tail -c 300 gpurun_out/final/bench_n2_rehearsal.json; tail -3 gpurun_out/final/bench_n2_rehearsal.err
timeout -k 10 300 python -u scripts/strong_probe.py synth1m_256 1,2,3,4,6,8 fused || exit 1
