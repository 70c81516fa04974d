# A/B/C...: several builds of the C-ABI (LIBS = space-separated label=path.so[,VAR=VALUE...]) on WORKLOADS,
# alternating per repetition on one box; one line per run with the aggregation kernel, the
# standalone encode, the pipelined step's kernel and the step time (bench events)
set -u -o pipefail
mkdir -p gpurun_out
WL=${WORKLOADS:-synth1m_256}
for rep in $(seq ${REPS:-2}); do
  for w in $WL; do
    for lp in $LIBS; do
      lab=${lp%%=*}; rest=${lp#*=}; lib=${rest%%,*}; envs=""; [ "$rest" != "$lib" ] && envs=${rest#*,}
      env ${envs//,/ } FLEET_CODEC_LIB=$PWD/$lib timeout -k 10 300 python bench.py --workload $w --extras= --no-cpu-baseline --no-e2e \
        --no-strong-block --steps ${STEPS:-20} --warmup 3 > gpurun_out/abm.json 2>gpurun_out/abm.err || { tail -5 gpurun_out/abm.err; exit 1; }
      python3 -c "
import json; r=json.loads(open('gpurun_out/abm.json').read().strip().splitlines()[-1])
k=r['kernels']; print('$lab', '$w', 'update', round(k['k_update_ms']*1e3,1), 'us  encode', round(k['k_encode_f32_ms']*1e3,1), 'us  fused', round(r['roofline']['kernel_ms']*1e3,1), 'us  step', round(r['ms_per_step']*1e3,1), 'us', flush=True)"
    done
  done
done
