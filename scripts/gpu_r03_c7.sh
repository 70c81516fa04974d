set -u
EXTRA_TESTS= WORKLOADS="synth1m_256 cifar10_256 mnist64" bash scripts/gpu_ab_quick.sh > gpurun_out/c7_ab.log 2>&1; echo "ab rc=$?"; tail -16 gpurun_out/c7_ab.log
bash scripts/gpu_kardam_plans.sh > gpurun_out/c7_kardam.log 2>&1; echo "kardam rc=$?"; cat gpurun_out/c7_kardam.log
