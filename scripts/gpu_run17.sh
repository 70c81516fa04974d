set -u
mkdir -p gpurun_out/r17
O=gpurun_out/r17
timeout -k 10 900 python -m pytest tests -m gpu -q -x -k "model" > $O/pytest_model.log 2>&1; echo "model rc=$?"; tail -15 $O/pytest_model.log
timeout -k 10 600 python -m pytest tests -m gpu -q -x > $O/pytest_gpu.log 2>&1; tail -2 $O/pytest_gpu.log
