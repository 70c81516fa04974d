# profile pass: kernel trace + stats per workload; FETCH_SIZE / WRITE_SIZE / SQ PMC passes; summaries
# usage: bash scripts/gpu_profile.sh TAG [WORKLOADS...]   (default: synth1m_256 cifar10_256 mnist64)
set -u
TAG=${1:-r02}; shift || true
WL=${*:-"synth1m_256 cifar10_256 mnist64"}
O=${OUTROOT:-$PWD/gpurun_out}/$TAG; mkdir -p $O
R=$PWD
export TMPDIR=/tmp
B="--extras= --no-cpu-baseline --no-e2e --no-strong-block"
for W in $WL; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_$W -o run -- python3 $R/bench.py --workload $W $B --steps 100 --warmup 3 > $O/trace_$W.log 2>&1 &&
  timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch_$W -o run -- python3 $R/bench.py --workload $W $B --steps 5 --warmup 1 > $O/fetch_$W.log 2>&1 &&
  timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/write_$W -o run -- python3 $R/bench.py --workload $W $B --steps 5 --warmup 1 > $O/write_$W.log 2>&1 &&
  timeout -s KILL 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_BUSY_CU_CYCLES SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE --output-format csv -d $O/sq_$W -o run -- python3 $R/bench.py --workload $W $B --steps 5 --warmup 1 > $O/sq_$W.log 2>&1 || exit 1
  echo "$W profiled"
done
# element-clients per launch of each workload (M * n_up)
ec() { python3 -c "import sys; sys.path.insert(0,'$R'); import bench; from fleet_amd.layouts import LAYOUTS; l,m,_=bench.WORKLOADS['$1']; print(m*LAYOUTS[l].n_up)"; }
TR=""; SQ=""
for W in $WL; do TR="$TR $W=$O/trace_$W,$O/fetch_$W,$O/write_$W"; SQ="$SQ $W=$O/sq_$W:$(ec $W)"; done
python3 scripts/pmc_summary.py $O/traffic.json $TR > /dev/null && echo traffic ok
python3 scripts/sq_summary.py $O/sq.json $SQ > /dev/null && echo sq ok
for W in $WL; do grep '^{' $O/trace_$W.log | tail -1 | cut -c1-150; done
