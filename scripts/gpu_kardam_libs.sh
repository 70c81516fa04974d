# Kardam's side outputs per library build (LIBS = "label=path.so[,VAR=VALUE...] ...") and workload
# (WORKLOADS): scripts/kardam_ab.py under rocprofv3 --kernel-trace --stats, the
# per-kernel averages of the plain update, the update with side outputs and the reduce
set -u -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=${OUT:-gpurun_out/klibs}; mkdir -p $O
for W in ${WORKLOADS:-mnist64 cifar10_256 synth1m_256}; do
  for lp in $LIBS; do
    lab=${lp%%=*}; rest=${lp#*=}; lib=${rest%%,*}; envs=""; [ "$rest" != "$lib" ] && envs=${rest#*,}
    env ${envs//,/ } FLEET_CODEC_LIB=$PWD/$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/${lab}_$W -o run -- python3 scripts/kardam_ab.py $W > $O/${lab}_$W.log 2>&1 || { tail -5 $O/${lab}_$W.log; exit 1; }
    python3 -c "
import csv
for r in csv.DictReader(open('$O/${lab}_$W/run_kernel_stats.csv')):
    n = r['Name']
    if 'k_update' in n or 'k_kardam_reduce' in n or 'k_kardam_finish' in n:
        print('%-8s %-12s %-44s calls %4s avg %9.1f us' % ('$lab', '$W', n.split('(')[0].replace('void fleet::', '').replace('fleet::', ''),
                                                   r['Calls'], float(r['AverageNs']) / 1e3), flush=True)
"
  done
done
