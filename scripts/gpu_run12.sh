set -u
mkdir -p gpurun_out/r12
R=$PWD
O=$R/gpurun_out/r12
export TMPDIR=/tmp
timeout -k 10 120 ./scripts/ubench_tiled > $O/ubench_tiled.log 2>&1 && cat $O/ubench_tiled.log &&
timeout -k 10 600 python -m pytest tests -m gpu -q -x > $O/pytest_gpu.log 2>&1; tail -3 $O/pytest_gpu.log
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY --output-format csv -d $O/pmc_mnist -o run -- python3 $R/bench.py --workload mnist64 --extras= --no-cpu-baseline --no-e2e --steps 5 --warmup 1 > $O/pmc_mnist.log 2>&1; echo pmc rc=$?
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY --output-format csv -d $O/pmc_s1m -o run -- python3 $R/bench.py --workload synth1m_256 --extras= --no-cpu-baseline --no-e2e --steps 3 --warmup 1 > $O/pmc_s1m.log 2>&1; echo pmc rc=$?
