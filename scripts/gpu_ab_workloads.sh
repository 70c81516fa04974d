# A/B: ab/libfleetcodec_prev.so (A) vs fleet_amd/libfleetcodec.so (B) on WORKLOADS (default the four
# single-GPU bench workloads), alternating, same box; prints aggregation / encode kernel times and step time
set -u
WL=${WORKLOADS:-"mnist64 cifar10_256 synth1m_256 synth4m_4096"}
one() { # $1 = label, $2 = workload, rest = env
  local lab=$1 w=$2; shift 2
  env "$@" timeout -k 10 300 python bench.py --workload $w --extras= --no-cpu-baseline --no-e2e --no-strong-block --steps ${STEPS:-20} --warmup 3 > gpurun_out/abw.json 2>/dev/null || exit 1
  python3 -c "
import json; r=json.loads(open('gpurun_out/abw.json').read().strip().splitlines()[-1])
print('$lab', '$w', 'update', round(r['kernels']['k_update_ms']*1e3,1), 'us  encode', round(r['kernels']['k_encode_f32_ms']*1e3,1), 'us  step', round(r['ms_per_step']*1e3,1), 'us  fused', round(r['roofline']['kernel_ms']*1e3,1), 'us  sequential', round(r['sequential']['ms_per_step']*1e3,1))"
}
for rep in 1 2; do
  for w in $WL; do
    one A $w FLEET_CODEC_LIB=$PWD/ab/libfleetcodec_prev.so
    one B $w A=1
  done
done
