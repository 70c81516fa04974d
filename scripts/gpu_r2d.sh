# SQ counters of the stream update kernel (VALU / LDS issue, bank conflicts)
set -u
O=gpurun_out/r2d; mkdir -p $O
export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CU_CYCLES SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_WAVES SQ_WAIT_INST_LDS --output-format csv -d $O/pmc1 -o run -- python3 bench.py --workload synth1m_256 --extras= --no-cpu-baseline --no-e2e --steps 3 --warmup 1 > $O/pmc1.log 2>&1; echo "pmc1 rc=$?"
timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU SQ_WAIT_ANY SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_ANY --output-format csv -d $O/pmc2 -o run -- python3 bench.py --workload synth1m_256 --extras= --no-cpu-baseline --no-e2e --steps 3 --warmup 1 > $O/pmc2.log 2>&1; echo "pmc2 rc=$?"
