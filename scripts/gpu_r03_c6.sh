set -u
timeout -k 10 300 python -u -m pytest -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_kardam_fused.py tests/test_gpu_model_state.py tests/test_oracle_golden.py -s > gpurun_out/c6_tests.log 2>&1; echo "tests rc=$?"; tail -12 gpurun_out/c6_tests.log
EXTRA_TESTS= WORKLOADS="synth1m_256" bash scripts/gpu_ab_quick.sh > gpurun_out/c6_ab.log 2>&1; echo "ab rc=$?"; tail -30 gpurun_out/c6_ab.log
