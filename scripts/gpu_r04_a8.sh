# r04 a8: Kardam's pipelined form with the chunked finish kernel (host adds the chunk sums)
set -u
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
O=${OUTROOT:-$GRAFT_REPO_ROOT/gpurun_out}/a8; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_kardam_fused.py tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread -k "kardam or keep_slots" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
OUT=$O/klibs LIBS="head=ab/libhead.so tree=fleet_amd/libfleetcodec.so" WORKLOADS="mnist64" bash scripts/gpu_kardam_libs.sh || exit 1
