# round-1 profile pass: bench + kernel trace per workload, FETCH/WRITE PMC passes
set -u
mkdir -p gpurun_out/r01
R=$PWD
O=$R/gpurun_out/r01
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests -m gpu -q -x > $O/pytest_gpu.log 2>&1 && tail -2 $O/pytest_gpu.log &&
timeout -k 10 300 python bench.py > $O/bench_default.log 2>&1 && tail -1 $O/bench_default.log | cut -c1-600 &&
for W in mnist64 cifar10_256 synth1m_256; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_$W -o run -- python3 $R/bench.py --workload $W --extras= --no-cpu-baseline --steps 20 --warmup 3 > $O/trace_$W.log 2>&1 &&
  timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch_$W -o run -- python3 $R/bench.py --workload $W --extras= --no-cpu-baseline --steps 5 --warmup 1 > $O/fetch_$W.log 2>&1 &&
  timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/write_$W -o run -- python3 $R/bench.py --workload $W --extras= --no-cpu-baseline --steps 5 --warmup 1 > $O/write_$W.log 2>&1 || exit 1
  echo "$W profiled"
done &&
python scripts/pmc_summary.py $O/traffic.json mnist64=$O/trace_mnist64,$O/fetch_mnist64,$O/write_mnist64 cifar10_256=$O/trace_cifar10_256,$O/fetch_cifar10_256,$O/write_cifar10_256 synth1m_256=$O/trace_synth1m_256,$O/fetch_synth1m_256,$O/write_synth1m_256 > /dev/null &&
cat $O/traffic.json
