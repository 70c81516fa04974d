# r04 a13: the Kardam stream form: a5 HEAD (k_update<1, true>) against the tree (update_lane, two
# clients per trip) and one client per trip with / without the 6-wave register cap, alternating
set -u
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
O=${OUTROOT:-$GRAFT_REPO_ROOT/gpurun_out}/a13; mkdir -p $O
for r in 1 2; do
  OUT=$O/klibs$r LIBS="head=ab/libhead.so tree=fleet_amd/libfleetcodec.so kd1t6=ab/libkd1t6.so kd1t1=ab/libkd1t1.so" WORKLOADS="synth1m_256" bash scripts/gpu_kardam_libs.sh || exit 1
done
