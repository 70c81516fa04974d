set -u
mkdir -p gpurun_out/r16
O=gpurun_out/r16
timeout -k 10 120 ./scripts/ubench_tiled > $O/ubench_tiled.log 2>&1 && cat $O/ubench_tiled.log &&
timeout -k 10 600 python -m pytest tests -m gpu -q -x > $O/pytest_gpu.log 2>&1; tail -2 $O/pytest_gpu.log
