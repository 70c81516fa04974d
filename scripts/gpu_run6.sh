set -u
mkdir -p gpurun_out
R=$PWD
export TMPDIR=/tmp
timeout -k 10 900 python -m pytest tests -m gpu -q -rf -x > gpurun_out/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -15 gpurun_out/pytest_gpu.log
if [ $rc -le 1 ]; then
  timeout -k 10 300 python bench.py --steps 20 --warmup 3 --cpu-budget 5 > gpurun_out/bench.log 2>&1; echo "bench rc=$?"
  python -c "
import json
d=json.loads(open('gpurun_out/bench.log').read().strip().splitlines()[-1])
print('main', d['value'], d['ms_per_step'], d['kernels'], d['roofline']['frac'])
print({k:(round(v['gib_s'],1),round(v['update_kernel_ms'],3),round(v['encode_kernel_ms'],3), round(v['update_gbs'],1)) for k,v in d['extra'].items()})
print(d['cpu_baseline'])
"
  FLEET_UPDATE_MODE=tiled timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --workload cifar10_256 --extras= > gpurun_out/bench_cifar_tiled.log 2>&1; echo "cifar tiled rc=$?"; tail -1 gpurun_out/bench_cifar_tiled.log | cut -c1-300
  timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_LDS SQ_INSTS_SALU --output-format csv -d $R/gpurun_out/pmc6 -o run -- python $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --workload synth1m_256 --extras= > gpurun_out/pmc6.log 2>&1; echo "pmc rc=$?"
fi
