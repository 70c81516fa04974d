set -u
mkdir -p gpurun_out
R=$PWD
export TMPDIR=/tmp
timeout -k 10 900 python -m pytest tests -m gpu -q -rf -x > gpurun_out/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -5 gpurun_out/pytest_gpu.log
if [ $rc -le 1 ]; then
  for TG in 16 32 64; do
    FLEET_TILE_G=$TG timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --extras= > gpurun_out/bench_tg$TG.log 2>&1; echo "tg$TG rc=$?"
    python -c "
import json
d=json.loads(open('gpurun_out/bench_tg$TG.log').read().strip().splitlines()[-1])
print('TG=$TG', round(d['value'],1), round(d['ms_per_step']*1e3,1),'us', {k:round(v,4) for k,v in d['kernels'].items()})
"
  done
  for K in 1 2; do
    FLEET_UPDATE_K=$K timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --workload synth1m_256 --extras=cifar10_256 > gpurun_out/bench_s1m_K$K.log 2>&1; echo "K$K rc=$?"
    python -c "
import json
d=json.loads(open('gpurun_out/bench_s1m_K$K.log').read().strip().splitlines()[-1])
print('K=$K', round(d['value'],1), d['ms_per_step'], {k:round(v,4) for k,v in d['kernels'].items()}, {k:(round(v['gib_s'],1),round(v['update_kernel_ms'],3),round(v['encode_kernel_ms'],3)) for k,v in d['extra'].items()})
"
  done
fi
