# r04 a28: the tiles' Kardam side outputs with one D stage per lane (ab/libtkd.so) against the tree
# (one per item): the Kardam tests on the new build, then the A/B on cifar10_256 / cifar100_1024
set -u
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
O=${OUTROOT:-$GRAFT_REPO_ROOT/gpurun_out}/a28; mkdir -p $O
FLEET_CODEC_LIB=$PWD/ab/libtkd.so timeout -k 10 400 python -u -m pytest tests/test_gpu_kardam_fused.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for r in 1 2; do
  OUT=$O/klibs$r LIBS="tree=fleet_amd/libfleetcodec.so tkd=ab/libtkd.so" WORKLOADS="cifar10_256 cifar100_1024" bash scripts/gpu_kardam_libs.sh || exit 1
done
