# r04 a19: the Kardam tests on the tree (late ladder rungs in its stream form); the CIFAR tiles' serial phase at issue priority 2 (ab/libtp2.so) against the tree, alternating
set -u
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
O=${OUTROOT:-$GRAFT_REPO_ROOT/gpurun_out}/a19; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_kardam_fused.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
LIBS="base=fleet_amd/libfleetcodec.so tp2=ab/libtp2.so" REPS=3 WORKLOADS="cifar10_256 cifar100_1024" STEPS=20 bash scripts/gpu_ab_multi.sh > $O/tile_p2prio.txt 2>&1 || { tail -5 $O/tile_p2prio.txt; exit 1; }
cat $O/tile_p2prio.txt
