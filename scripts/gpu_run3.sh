set -u
mkdir -p gpurun_out
R=$PWD
timeout -k 10 900 python -m pytest tests -m gpu -q -rf -x > gpurun_out/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -15 gpurun_out/pytest_gpu.log
if [ $rc -le 1 ]; then
  export TMPDIR=/tmp
  for K in 1 2 4; do
    FLEET_UPDATE_K=$K timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --workload synth1m_256 --extras cifar10_256 > gpurun_out/bench_K$K.log 2>&1; echo "bench K=$K rc=$?"
    python -c "
import json,sys
d=json.loads(open('gpurun_out/bench_K$K.log').read().strip().splitlines()[-1])
print('K=$K', d['value'], d['ms_per_step'], d['kernels'], {k:(v['gib_s'],v['update_kernel_ms'],v['encode_kernel_ms']) for k,v in d['extra'].items()})
"
  done
  timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof4 -o run -- python $R/bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/bench_prof.log 2>&1; echo "rocprof rc=$?"
  tail -1 gpurun_out/bench_prof.log | cut -c1-600
  cat gpurun_out/prof4/run_kernel_stats.csv | cut -c1-200
fi
