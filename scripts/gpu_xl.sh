# q_xl consumer: digest + pipe-variant parity, then same-box A/B bench
set -u
O=gpurun_out/xl; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -k "digest or pipe or update or tile" > $O/pytest.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -3 $O/pytest.log; [ $rc -ne 0 ] && exit 1
bash scripts/gpu_ab.sh
