set -u
timeout -k 10 300 python -u -m pytest -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_kardam_fused.py tests/test_gpu_full_size.py -k "kardam or ingress" > gpurun_out/c8_tests.log 2>&1; echo "tests rc=$?"; tail -3 gpurun_out/c8_tests.log
bash scripts/gpu_kardam_plans.sh > gpurun_out/c8_kardam.log 2>&1 || exit 1
FLEET_KARDAM_PIPE_NW=5 WORKLOADS=mnist64 bash scripts/gpu_kardam_plans.sh > gpurun_out/c8_kardam5.log 2>&1 || exit 1
for w in mnist64 cifar10_256 synth1m_256; do echo "== $w"; python3 -c "
import csv
for r in csv.DictReader(open('gpurun_out/kplan_$w/run_kernel_stats.csv')):
    n=r['Name']
    if 'k_update' in n or 'k_kardam' in n:
        print('%-40s calls %4s avg %8.1f us' % (n.split('(')[0].replace('void fleet::',''), r['Calls'], float(r['AverageNs'])/1e3))
"; done
