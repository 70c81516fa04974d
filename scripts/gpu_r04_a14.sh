# r04 a14: the Kardam stream form, one client per trip (the tree) against a5 HEAD (k_update<1, true>)
# and the tree with the issue-priority ladder (ab/libkdlad.so), alternating; the Kardam GPU tests
set -u
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
O=${OUTROOT:-$GRAFT_REPO_ROOT/gpurun_out}/a14; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_kardam_fused.py tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread -k "kardam or keep_slots" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for r in 1 2; do
  OUT=$O/klibs$r LIBS="head=ab/libhead.so tree=fleet_amd/libfleetcodec.so kdlad=ab/libkdlad.so" WORKLOADS="synth1m_256" bash scripts/gpu_kardam_libs.sh || exit 1
done
