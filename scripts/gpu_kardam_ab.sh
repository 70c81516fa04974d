# A/B of the fused Kardam update (k_update<1, true>) on synth1m_256: ab/libfleetcodec_prev.so (A)
# against the tree's library (B), each under rocprofv3 --kernel-trace --stats (scripts/kardam_ab.py)
set -u
export TMPDIR=/tmp
for lab in A B; do
  if [ $lab = A ]; then L=$PWD/ab/libfleetcodec_prev.so; else L=$PWD/fleet_amd/libfleetcodec.so; fi
  FLEET_CODEC_LIB=$L timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/kab_$lab -o run -- python3 scripts/kardam_ab.py > gpurun_out/kab_$lab.log 2>&1 || exit 1
  echo "$lab"; grep -h "k_update<1, true\|k_kardam\|k_update_mixed\|k_update<1, false" gpurun_out/kab_$lab/run_kernel_stats.csv | cut -d, -f1-4
done
