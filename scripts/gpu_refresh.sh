# full GPU test suite, profile pass (traces + PMC) and the default bench line
set -u
O=gpurun_out/refresh; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -2 $O/pytest.log; [ $rc -ne 0 ] && exit 1
bash scripts/gpu_profile2.sh refresh || exit 1
cp gpurun_out/refresh/traffic.json profiles/r01/traffic.json
timeout -k 10 600 python bench.py > $O/bench_default.json 2> $O/bench_default.err; echo "bench rc=$?"; tail -c 600 $O/bench_default.json
