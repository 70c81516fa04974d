# r04 a23: the value's N = 1 / 2 windows with the fused step's update blocks a value per lane
# (grid=lanes: 3x the waves at a third of the work) against the group-per-lane grid; fused-step tests
set -u
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
O=${OUTROOT:-$GRAFT_REPO_ROOT/gpurun_out}/a23; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_fused_step.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for r in 1 2; do
  timeout -k 10 300 python3 scripts/strong_probe.py synth1m_256 1,2 fused > $O/plain$r.log 2>&1 || { tail -5 $O/plain$r.log; exit 1; }
  grep speedup $O/plain$r.log
  FLEET_EXPERIMENTS=grid=lanes timeout -k 10 300 python3 scripts/strong_probe.py synth1m_256 1,2 fused > $O/lanes$r.log 2>&1 || { tail -5 $O/lanes$r.log; exit 1; }
  grep speedup $O/lanes$r.log
done
