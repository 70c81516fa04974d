# Copy a profile pass (scripts/gpu_profile.sh TAG) from gpurun_out/ into profiles/TAG/ under the
# names the bench and DESIGN.md cite: <workload>_{kernel_stats,fetch_size,write_size,sq}.csv,
# traffic.json, sq.json.  usage: bash scripts/collect_profiles.sh TAG [SRC_DIR]
set -eu
TAG=$1; SRC=${2:-gpurun_out/$TAG}; DST=profiles/$TAG
mkdir -p $DST
for d in $SRC/trace_*; do
  [ -d $d ] || continue
  W=${d##*/trace_}
  cp $d/run_kernel_stats.csv $DST/${W}_kernel_stats.csv
  [ -f $SRC/fetch_$W/run_counter_collection.csv ] && cp $SRC/fetch_$W/run_counter_collection.csv $DST/${W}_fetch_size.csv
  [ -f $SRC/write_$W/run_counter_collection.csv ] && cp $SRC/write_$W/run_counter_collection.csv $DST/${W}_write_size.csv
  [ -f $SRC/sq_$W/run_counter_collection.csv ] && cp $SRC/sq_$W/run_counter_collection.csv $DST/${W}_sq.csv
  grep '^{' $SRC/trace_$W.log | tail -1 > $DST/bench_${W}_under_rocprof.json || true
done
for f in traffic.json sq.json; do [ -f $SRC/$f ] && cp $SRC/$f $DST/$f; done
ls $DST
