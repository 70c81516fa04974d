# Base64 decode: bytes 1 and 2 by SDWA moves vs v_bfe (parity of the variant first)
set -u
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
FLEET_CODEC_LIB=$PWD/ab/lib_sdwa.so timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_fused_step.py tests/test_gpu_full_size.py > gpurun_out/d16_tests.log 2>&1; rc=$?; tail -1 gpurun_out/d16_tests.log; [ $rc = 0 ] || exit 1
LIBS="base=ab/lib_base.so sdwa=ab/lib_sdwa.so" REPS=3 WORKLOADS="synth1m_256 cifar10_256" bash scripts/gpu_ab_multi.sh
