# parity of the current build, then the A/B bench
set -u
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -k "update or digest" > gpurun_out/abt_pytest.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/abt_pytest.log; [ $rc -ne 0 ] && exit 1
bash scripts/gpu_ab.sh
