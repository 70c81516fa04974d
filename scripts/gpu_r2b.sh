# instruction-cost microbenchmark + VALU counters of the stream kernel
set -u
O=gpurun_out/r2b; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 120 ./scripts/ubench3 > $O/ubench3.txt 2>&1; rc=$?; echo "ubench rc=$rc"; cat $O/ubench3.txt; [ $rc -ge 124 ] && exit $rc
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INST_CYCLES_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CU_CYCLES SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_WAVES --output-format csv -d $O/pmc_sq -o run -- python3 bench.py --workload synth1m_256 --extras= --no-cpu-baseline --no-e2e --steps 3 --warmup 1 > $O/pmc_sq.log 2>&1; rc=$?; echo "pmc rc=$rc"
