# A/B of ab/libfleetcodec_prev.so (A) vs fleet_amd/libfleetcodec.so (B) on one workload under
# several environment settings (ENVS, space-separated items of comma-joined VAR=VALUE; "-" = none)
set -u
W=${W:-synth1m_256}
for e in ${ENVS:-"-"}; do
  for lab in A B; do
    if [ $lab = A ]; then L=FLEET_CODEC_LIB=$PWD/ab/libfleetcodec_prev.so; else L=B=1; fi
    E=${e//,/ }; [ "$E" = "-" ] && E=NONE=1
    env $L $E timeout -k 10 300 python bench.py --workload $W --extras= --no-cpu-baseline --no-e2e --no-strong-block --steps ${STEPS:-20} --warmup 3 > gpurun_out/abe.json 2>/dev/null || exit 1
    python3 -c "
import json; r=json.loads(open('gpurun_out/abe.json').read().strip().splitlines()[-1])
k=r['kernels']; print('$lab', '$W', '$e', 'update', round(k['k_update_ms']*1e3,1), 'us  encode', round(k['k_encode_f32_ms']*1e3,1), 'us  step', round(r['ms_per_step']*1e3,1), 'us  fused', round(r['roofline']['kernel_ms']*1e3,1), 'us  kernel', r['roofline']['kernel'])"
  done
done
