set -u
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_fused_step.py tests/test_gpu_full_size.py > gpurun_out/c1_tests.log 2>&1; rc=$?; tail -3 gpurun_out/c1_tests.log; [ $rc = 0 ] || exit 1
LIBS="head=ab/lib_head.so v00=ab/lib_v00.so v10=ab/lib_v10.so v01=ab/lib_v01.so v11=ab/lib_v11.so" REPS=2 WORKLOADS=synth1m_256 bash scripts/gpu_ab_multi.sh
