# r04 a5: the new Kardam stream form (k_update_mixed<256, true>) and keep-slot tests, the Kardam
# A/B (HEAD library = k_update<1, true> + the old reduce; the tree; the tree without the
# register cap), the issue-priority ladder A/B, and the MNIST-64 phase timestamps
set -u
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=${OUTROOT:-$GRAFT_REPO_ROOT/gpurun_out}/a5; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_kardam_fused.py tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread -k "kardam or keep_slots" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
OUT=$O/klibs LIBS="head=ab/libhead.so tree=fleet_amd/libfleetcodec.so kd1=ab/libkd1.so" WORKLOADS="synth1m_256" bash scripts/gpu_kardam_libs.sh || exit 1
OUT=$O/klibs LIBS="head=ab/libhead.so tree=fleet_amd/libfleetcodec.so" WORKLOADS="mnist64 cifar10_256" bash scripts/gpu_kardam_libs.sh || exit 1
LIBS="base=fleet_amd/libfleetcodec.so ladder=ab/libladder.so" REPS=3 WORKLOADS="synth1m_256" STEPS=20 bash scripts/gpu_ab_multi.sh || exit 1
timeout -k 10 120 ./scripts/ubench_tiled > $O/ubench_tiled.log 2>&1 || exit 1
tail -20 $O/ubench_tiled.log
