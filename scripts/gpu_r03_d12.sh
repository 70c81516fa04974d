# strong-scaling windows of synth1m_256 (N = 2..8): launch form of the pipelined step per window size
set -u
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
P="timeout -k 10 200 python -u scripts/strong_probe.py synth1m_256 2,3,4,6,8 fused"
echo "== default"; $P || exit 1
echo "== stream"; FLEET_UPDATE_MODE=stream $P || exit 1
for tg in 64 32 16; do echo "== tiled $tg"; FLEET_UPDATE_MODE=tiled FLEET_TILE_G=$tg $P || exit 1; done
echo "== tiled 64 inline"; FLEET_UPDATE_MODE=tiled FLEET_TILE_G=64 FLEET_FUSED_TILE_INLINE=1 $P || exit 1
echo "== tiled 32 inline"; FLEET_UPDATE_MODE=tiled FLEET_TILE_G=32 FLEET_FUSED_TILE_INLINE=1 $P || exit 1
echo "== tiled 64 mix"; FLEET_UPDATE_MODE=tiled FLEET_TILE_G=64 FLEET_FUSED_TILE_MIX=1 $P || exit 1
