set -u
export TMPDIR=/tmp
EXTRA_TESTS= WORKLOADS="cifar10_256 cifar100_1024" bash scripts/gpu_ab_quick.sh > gpurun_out/c10_ab.log 2>&1; echo "ab rc=$?"; tail -9 gpurun_out/c10_ab.log
B="--extras= --no-cpu-baseline --no-e2e --no-strong-block"
for lab in A B; do
  if [ $lab = A ]; then L=$PWD/ab/libfleetcodec_prev.so; else L=$PWD/fleet_amd/libfleetcodec.so; fi
  FLEET_CODEC_LIB=$L timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/c10_fetch_$lab -o run -- python3 bench.py --workload cifar10_256 $B --steps 5 --warmup 1 > gpurun_out/c10_fetch_$lab.log 2>&1 || exit 1
  FLEET_CODEC_LIB=$L timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/c10_write_$lab -o run -- python3 bench.py --workload cifar10_256 $B --steps 5 --warmup 1 > gpurun_out/c10_write_$lab.log 2>&1 || exit 1
  python3 scripts/pmc_summary.py gpurun_out/c10_traffic_$lab.json cifar10_256=gpurun_out/none,gpurun_out/c10_fetch_$lab,gpurun_out/c10_write_$lab > /dev/null
  python3 -c "
import json; k=json.load(open('gpurun_out/c10_traffic_$lab.json'))['workloads']['cifar10_256']
for n, e in sorted(k.items()):
    if 'hbm_bytes' in e: print('$lab', n, 'hbm bytes per launch %.1f MB' % (e['hbm_bytes'] / 1e6))
"
done
