# inline encode in the fused step: parity (fused step + full size), then A/B against HEAD and the separate-block form
set -u
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_fused_step.py tests/test_gpu_full_size.py tests/test_gpu_parity.py > gpurun_out/d2_tests.log 2>&1; rc=$?; tail -3 gpurun_out/d2_tests.log; [ $rc = 0 ] || exit 1
LIBS="head=ab/lib_head.so inl=ab/lib_inl.so sep=ab/lib_inl.so,FLEET_FUSED_INLINE=0 v00=ab/lib_v00.so" REPS=3 WORKLOADS=synth1m_256 bash scripts/gpu_ab_multi.sh
