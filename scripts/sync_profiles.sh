# copy a profile pass (scripts/gpu_profile2.sh TAG, run through gpurun) into profiles/r01
set -eu
TAG=${1:-refresh}; I=gpurun_out/$TAG; O=profiles/r01
for W in mnist64 cifar10_256 synth1m_256; do
  cp $I/trace_$W/run_kernel_stats.csv $O/${W}_kernel_stats.csv
  cp $I/fetch_$W/run_counter_collection.csv $O/${W}_fetch_size.csv
  cp $I/write_$W/run_counter_collection.csv $O/${W}_write_size.csv
  cp $I/sq_$W/run_counter_collection.csv $O/${W}_sq.csv
  grep '^{' $I/trace_$W.log | tail -1 > $O/bench_${W}_under_rocprof.json
done
cp $I/traffic.json $I/sq.json $O/
[ -f $I/bench_default.json ] && grep '^{' $I/bench_default.json | tail -1 > $O/bench_default.json
echo synced
