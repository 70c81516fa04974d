set -u
mkdir -p gpurun_out
timeout -k 10 120 ./scripts/ubench_chain > gpurun_out/ubench_chain.log 2>&1 && cat gpurun_out/ubench_chain.log &&
timeout -k 10 120 ./scripts/ubench_tiled > gpurun_out/ubench_tiled.log 2>&1 && cat gpurun_out/ubench_tiled.log &&
timeout -k 10 600 python -m pytest tests -m gpu -q -x > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] && timeout -k 10 300 python scripts/sweep_update.py mnist > gpurun_out/sweep_mnist.log 2>&1 && cat gpurun_out/sweep_mnist.log &&
timeout -k 10 300 python scripts/sweep_update.py cifar10 256 > gpurun_out/sweep_cifar.log 2>&1 && cat gpurun_out/sweep_cifar.log
