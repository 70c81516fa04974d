# r04 a24: the Kardam stream form at 7 / 8 waves per SIMD (ab/libkw7.so: 71 VGPRs + 16 B scratch;
# ab/libkw8.so: 64 VGPRs + 64 B scratch) against the tree's 6, alternating
set -u
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
O=${OUTROOT:-$GRAFT_REPO_ROOT/gpurun_out}/a24; mkdir -p $O
for r in 1 2; do
  OUT=$O/klibs$r LIBS="tree=fleet_amd/libfleetcodec.so kw7=ab/libkw7.so kw8=ab/libkw8.so" WORKLOADS="synth1m_256" bash scripts/gpu_kardam_libs.sh || exit 1
done
