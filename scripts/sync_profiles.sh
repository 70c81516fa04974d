# copy a profile pass (scripts/gpu_profile.sh TAG, run through gpurun) into profiles/<round>
# usage: bash scripts/sync_profiles.sh TAG [ROUND] [WORKLOADS...]
set -eu
TAG=${1:-r02}; RND=${2:-r02}; shift 2 || shift $#
WL=${*:-"synth1m_256 cifar10_256 mnist64"}
I=gpurun_out/$TAG; O=profiles/$RND; mkdir -p $O
for W in $WL; do
  cp $I/trace_$W/run_kernel_stats.csv $O/${W}_kernel_stats.csv
  cp $I/fetch_$W/run_counter_collection.csv $O/${W}_fetch_size.csv
  cp $I/write_$W/run_counter_collection.csv $O/${W}_write_size.csv
  cp $I/sq_$W/run_counter_collection.csv $O/${W}_sq.csv
  grep '^{' $I/trace_$W.log | tail -1 > $O/bench_${W}_under_rocprof.json
done
cp $I/traffic.json $I/sq.json $O/
if [ -f $I/bench_default.json ]; then grep '^{' $I/bench_default.json | tail -1 > $O/bench_default.json; fi
echo synced
