# r04 a10: the issue-priority ladder in the CIFAR tiles (ab/libtladder.so, FLEET_TILE_LADDER=1)
# against the tree, alternating on one box
set -u
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
O=${OUTROOT:-$GRAFT_REPO_ROOT/gpurun_out}/a10; mkdir -p $O
LIBS="base=fleet_amd/libfleetcodec.so tladder=ab/libtladder.so" REPS=3 WORKLOADS="cifar10_256 cifar100_1024" STEPS=20 bash scripts/gpu_ab_multi.sh > $O/tile_ladder.txt 2>&1 || { tail -5 $O/tile_ladder.txt; exit 1; }
cat $O/tile_ladder.txt
