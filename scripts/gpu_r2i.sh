set -u
timeout -k 10 300 python -u -m pytest tests/test_updater.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r2i_updater.log 2>&1; rc=$?; echo "updater rc=$rc"; tail -2 gpurun_out/r2i_updater.log; [ $rc -ge 124 ] && exit $rc
bash scripts/gpu_profile2.sh r01c || exit 1
timeout -k 10 400 python bench.py > gpurun_out/r01c/bench_default.json 2> gpurun_out/r01c/bench_default.err; echo "bench rc=$?"
