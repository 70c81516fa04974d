# profile pass: kernel trace + stats per workload; FETCH_SIZE / WRITE_SIZE / SQ PMC passes; summaries
set -u
TAG=${1:-r01}
O=$PWD/gpurun_out/$TAG; mkdir -p $O
R=$PWD
export TMPDIR=/tmp
for W in mnist64 cifar10_256 synth1m_256; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_$W -o run -- python3 $R/bench.py --workload $W --extras= --no-cpu-baseline --no-e2e --steps 20 --warmup 3 > $O/trace_$W.log 2>&1 &&
  timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch_$W -o run -- python3 $R/bench.py --workload $W --extras= --no-cpu-baseline --no-e2e --steps 5 --warmup 1 > $O/fetch_$W.log 2>&1 &&
  timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/write_$W -o run -- python3 $R/bench.py --workload $W --extras= --no-cpu-baseline --no-e2e --steps 5 --warmup 1 > $O/write_$W.log 2>&1 &&
  timeout -s KILL 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_BUSY_CU_CYCLES SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE --output-format csv -d $O/sq_$W -o run -- python3 $R/bench.py --workload $W --extras= --no-cpu-baseline --no-e2e --steps 5 --warmup 1 > $O/sq_$W.log 2>&1 || exit 1
  echo "$W profiled"
done
python3 scripts/pmc_summary.py $O/traffic.json mnist64=$O/trace_mnist64,$O/fetch_mnist64,$O/write_mnist64 cifar10_256=$O/trace_cifar10_256,$O/fetch_cifar10_256,$O/write_cifar10_256 synth1m_256=$O/trace_synth1m_256,$O/fetch_synth1m_256,$O/write_synth1m_256 > /dev/null && echo traffic ok
python3 scripts/sq_summary.py $O/sq.json mnist64=$O/sq_mnist64:1469504 cifar10_256=$O/sq_cifar10_256:80349952 synth1m_256=$O/sq_synth1m_256:268435456 > /dev/null && echo sq ok
for W in mnist64 cifar10_256 synth1m_256; do tail -1 $O/trace_$W.log | cut -c1-150; done
