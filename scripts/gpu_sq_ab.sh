# SQ counter passes for the aggregation kernel variants on one workload:
# A = ab/libfleetcodec_prev.so, B = fleet_amd/libfleetcodec.so, B with extra env (VARIANTS)
# usage: W=synth1m_256 bash scripts/gpu_sq_ab.sh   (writes gpurun_out/sqab/<label>_p<k>/)
set -u
W=${W:-synth1m_256}
O=gpurun_out/sqab; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_LDS"
P2="SQ_LDS_BANK_CONFLICT SQ_LDS_ADDR_CONFLICT SQ_LDS_DATA_FIFO_FULL SQ_LDS_CMD_FIFO_FULL SQ_LDS_UNALIGNED_STALL SQ_ACTIVE_INST_ANY SQ_INST_LEVEL_LDS SQ_LDS_IDX_ACTIVE"
P3="SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_MISC SQ_INSTS_SALU SQ_WAVES SQ_CYCLES SQ_WAIT_ANY"
for v in ${VARIANTS:-"A:FLEET_CODEC_LIB=$PWD/ab/libfleetcodec_prev.so" "B:X=1"}; do
  lab=${v%%:*}; env_=${v#*:}
  k=0
  for P in "$P1" "$P2" "$P3"; do
    k=$((k+1))
    env $env_ timeout -s KILL 120 rocprofv3 --pmc $P --output-format csv -d $O/${lab}_p$k -o run -- python3 bench.py --workload $W --extras= --no-cpu-baseline --no-e2e --no-strong-block --steps 3 --warmup 1 > $O/${lab}_p$k.log 2>&1 || exit 1
  done
  echo "$lab done"
done
