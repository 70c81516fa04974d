# r04 a9: Kardam A/B, alternating on one box (then the tile ladder A/B of a10): the a5 HEAD library (k_update<1, true>, the NW=8
# pipelined producers + reduce) against the tree (the plain-grid stream form; the pipelined form's
# p rows + chunked finish, its loads issued before the table copy)
set -u
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
O=${OUTROOT:-$GRAFT_REPO_ROOT/gpurun_out}/a9; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_kardam_fused.py tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread -k "kardam or keep_slots" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for r in 1 2 3; do
  OUT=$O/klibs$r LIBS="head=ab/libhead.so tree=fleet_amd/libfleetcodec.so" WORKLOADS="mnist64 synth1m_256 cifar10_256" bash scripts/gpu_kardam_libs.sh || exit 1
done

LIBS="base=fleet_amd/libfleetcodec.so tladder=ab/libtladder.so" REPS=3 WORKLOADS="cifar10_256 cifar100_1024" STEPS=20 bash scripts/gpu_ab_multi.sh > $O/tile_ladder.txt 2>&1 || { tail -5 $O/tile_ladder.txt; exit 1; }
cat $O/tile_ladder.txt
