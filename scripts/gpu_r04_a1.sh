# r04 a1: per-wave progress traces of the stream aggregation on configs[4]'s windows
# (scripts/ubench_window.hip), and the list of PMC counters on this box
set -u
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/a1; mkdir -p $O
timeout -k 10 120 rocprofv3 -L > $O/counters.txt 2>&1 || echo "counter list rc=$?"
timeout -k 10 120 ./scripts/ubench_window 349526 256,1024 mixed w4 > $O/trace.log 2>&1 || exit 1
timeout -k 10 120 ./scripts/ubench_window 349526 1024 plain w4 >> $O/trace.log 2>&1 || exit 1
timeout -k 10 120 ./scripts/ubench_window 174763 256,1024 mixed w8 >> $O/trace.log 2>&1 || exit 1
timeout -k 10 200 ./scripts/ubench_window 1398102 256,1024 mixed full >> $O/trace.log 2>&1 || exit 1
mv gpurun_out/window_*.bin $O/ 2>/dev/null
cat $O/trace.log
