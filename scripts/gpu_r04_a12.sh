# r04 a12: the Kardam A/B (a5 HEAD library against the tree, alternating) and the tile-ladder A/B
set -u
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
O=${OUTROOT:-$GRAFT_REPO_ROOT/gpurun_out}/a12; mkdir -p $O
for r in 1 2; do
  OUT=$O/klibs$r LIBS="head=ab/libhead.so tree=fleet_amd/libfleetcodec.so" WORKLOADS="mnist64 synth1m_256 cifar10_256" bash scripts/gpu_kardam_libs.sh || exit 1
done
LIBS="base=fleet_amd/libfleetcodec.so tladder=ab/libtladder.so" REPS=3 WORKLOADS="cifar10_256 cifar100_1024" STEPS=20 bash scripts/gpu_ab_multi.sh > $O/tile_ladder.txt 2>&1 || { tail -5 $O/tile_ladder.txt; exit 1; }
cat $O/tile_ladder.txt
