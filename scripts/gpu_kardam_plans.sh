# Kardam's side outputs on every launch plan: rocprofv3 kernel stats of scripts/kardam_ab.py per
# workload (TAG names the output dirs), summarised as per-kernel averages
set -u
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
TAG=${TAG:-kplan}
for W in ${WORKLOADS:-mnist64 cifar10_256 synth1m_256}; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_$W -o run -- python3 scripts/kardam_ab.py $W > gpurun_out/${TAG}_$W.log 2>&1 || exit 1
  echo "== $W"
  python3 -c "
import csv
for r in csv.DictReader(open('gpurun_out/${TAG}_$W/run_kernel_stats.csv')):
    n = r['Name']
    if 'k_update' in n or 'k_kardam' in n:
        print('%-42s calls %4s avg %8.1f us' % (n.split('(')[0].replace('void fleet::', '').replace('fleet::', ''),
                                                r['Calls'], float(r['AverageNs']) / 1e3))
"
done
