# r04 a22: the strong windows of the value at N = 3, 4, 6, 8 on the stream grid (plan override
# update=stream) against the planner's tiles -- with the ladder, does the stream grid win lower?
set -u
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
O=${OUTROOT:-$GRAFT_REPO_ROOT/gpurun_out}/a22; mkdir -p $O
for r in 1 2; do
  timeout -k 10 300 python3 scripts/strong_probe.py synth1m_256 1,3,4,6,8 fused > $O/tiles$r.log 2>&1 || { tail -5 $O/tiles$r.log; exit 1; }
  grep speedup $O/tiles$r.log
  FLEET_EXPERIMENTS=update=stream timeout -k 10 300 python3 scripts/strong_probe.py synth1m_256 3,4,6,8 fused > $O/stream$r.log 2>&1 || { tail -5 $O/stream$r.log; exit 1; }
  grep speedup $O/stream$r.log
done
