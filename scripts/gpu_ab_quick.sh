# correctness of the tree's library (the GPU suite's update/full-size tests), then the
# A/B of ab/libfleetcodec_prev.so (A) against it (B) on WORKLOADS (scripts/gpu_ab_workloads.sh)
set -u
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py tests/test_gpu_full_size.py tests/test_gpu_fused_step.py ${EXTRA_TESTS:-} \
  > gpurun_out/abq_tests.log 2>&1 || { tail -30 gpurun_out/abq_tests.log; exit 1; }
tail -1 gpurun_out/abq_tests.log
WORKLOADS=${WORKLOADS:-synth1m_256} STEPS=${STEPS:-20} bash scripts/gpu_ab_workloads.sh
