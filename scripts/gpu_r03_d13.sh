# strong windows: the new fused tile width rule; update alone at TG 32 / 64; value-per-lane stream grid at N = 2, 3
set -u
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_fused_step.py > gpurun_out/d13_tests.log 2>&1; rc=$?; tail -1 gpurun_out/d13_tests.log; [ $rc = 0 ] || exit 1
P="timeout -k 10 200 python -u scripts/strong_probe.py synth1m_256"
echo "== fused default"; $P 1,2,3,4,6,8 fused || exit 1
for tg in 32 64; do echo "== upd tiled $tg"; FLEET_UPDATE_MODE=tiled FLEET_TILE_G=$tg $P 6,8 upd || exit 1; done
echo "== fused stream mixed=2"; FLEET_UPDATE_MODE=stream FLEET_UPDATE_MIXED=2 FLEET_FUSED_PLAIN=0 $P 2,3 fused || exit 1
echo "== upd stream mixed=2"; FLEET_UPDATE_MODE=stream FLEET_UPDATE_MIXED=2 $P 2,3 upd || exit 1
echo "== upd default"; $P 2,3 upd || exit 1
