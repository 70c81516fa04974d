# r04 a21: the N = 2 window of the value (174,763 groups) on the tiles instead of the stream grid
# (plan override update=tiled) -- would a higher stream threshold help strong scaling at N = 2?
set -u
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
O=${OUTROOT:-$GRAFT_REPO_ROOT/gpurun_out}/a21; mkdir -p $O
for r in 1 2; do
  timeout -k 10 300 python3 scripts/strong_probe.py synth1m_256 1,2,3 fused > $O/stream$r.log 2>&1 || { tail -5 $O/stream$r.log; exit 1; }
  grep speedup $O/stream$r.log
  FLEET_EXPERIMENTS=update=tiled timeout -k 10 300 python3 scripts/strong_probe.py synth1m_256 2,3 fused > $O/tiled$r.log 2>&1 || { tail -5 $O/tiled$r.log; exit 1; }
  grep speedup $O/tiled$r.log
done
