set -u
mkdir -p gpurun_out
R=$PWD
export TMPDIR=/tmp
timeout -k 10 120 ./scripts/ubench2 > gpurun_out/ubench2.log 2>&1; echo "ubench2 rc=$?"; cat gpurun_out/ubench2.log
B="python $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --workload synth1m_256 --extras="
i=0
for P in "SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES" "FETCH_SIZE" "WRITE_SIZE" "GRBM_GUI_ACTIVE SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_SALU SQ_LDS_BANK_CONFLICT"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $P --output-format csv -d $R/gpurun_out/pmc$i -o run -- $B > gpurun_out/pmc$i.log 2>&1; echo "pmc$i rc=$?"
done
ls gpurun_out/pmc*/
