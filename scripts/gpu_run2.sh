set -u
mkdir -p gpurun_out
R=$PWD
timeout -k 10 120 ./scripts/ubench_valu > gpurun_out/ubench.log 2>&1; echo "ubench rc=$?"; cat gpurun_out/ubench.log
timeout -k 10 900 python -m pytest tests -m gpu -q -rf > gpurun_out/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -5 gpurun_out/pytest_gpu.log
if [ $rc -le 1 ]; then
  export TMPDIR=/tmp
  timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof -o run -- python $R/bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/bench_prof.log 2>&1; echo "rocprof rc=$?"
  tail -3 gpurun_out/bench_prof.log
  find gpurun_out/prof -name "*stats*" | head
fi
