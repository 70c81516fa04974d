# the fused step at 8 waves per SIMD (amdgpu_waves_per_eu, 64 VGPRs + 32 B of scratch) vs 7 (68 VGPRs)
set -u
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
FLEET_CODEC_LIB=$PWD/ab/lib_w8.so timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_fused_step.py > gpurun_out/d18_tests.log 2>&1; rc=$?; tail -1 gpurun_out/d18_tests.log; [ $rc = 0 ] || exit 1
LIBS="base=ab/lib_base.so w8=ab/lib_w8.so" REPS=3 WORKLOADS=synth1m_256 bash scripts/gpu_ab_multi.sh
