set -u
mkdir -p gpurun_out
timeout -k 10 120 ./scripts/ubench_tiled > gpurun_out/ubench_tiled.log 2>&1 && cat gpurun_out/ubench_tiled.log &&
timeout -k 10 600 python -m pytest tests -m gpu -q -x > gpurun_out/pytest_gpu.log 2>&1; tail -3 gpurun_out/pytest_gpu.log
