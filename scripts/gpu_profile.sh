# profile pass: kernel trace + stats per workload, FETCH_SIZE / WRITE_SIZE PMC passes, summary
set -u
TAG=${1:-r01}
mkdir -p gpurun_out/$TAG
R=$PWD
O=$R/gpurun_out/$TAG
export TMPDIR=/tmp
for W in mnist64 cifar10_256 synth1m_256; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_$W -o run -- python3 $R/bench.py --workload $W --extras= --no-cpu-baseline --no-e2e --steps 20 --warmup 3 > $O/trace_$W.log 2>&1 &&
  timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch_$W -o run -- python3 $R/bench.py --workload $W --extras= --no-cpu-baseline --no-e2e --steps 5 --warmup 1 > $O/fetch_$W.log 2>&1 &&
  timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/write_$W -o run -- python3 $R/bench.py --workload $W --extras= --no-cpu-baseline --no-e2e --steps 5 --warmup 1 > $O/write_$W.log 2>&1 || exit 1
  echo "$W profiled"
done
python scripts/pmc_summary.py $O/traffic.json mnist64=$O/trace_mnist64,$O/fetch_mnist64,$O/write_mnist64 cifar10_256=$O/trace_cifar10_256,$O/fetch_cifar10_256,$O/write_cifar10_256 synth1m_256=$O/trace_synth1m_256,$O/fetch_synth1m_256,$O/write_synth1m_256 > /dev/null && echo summary ok
for W in mnist64 cifar10_256 synth1m_256; do tail -1 $O/trace_$W.log | cut -c1-200; done
