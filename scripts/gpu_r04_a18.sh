# r04 a18: the ladder's rungs: quarters (the tree) against early (M/8, M/4, M/2: ab/libls1.so) and
# late (M/2, 3M/4, 7M/8: ab/libls2.so) rungs, alternating on synth1m_256 (aggregation alone and the
# fused step) and the Kardam stream form
set -u
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
O=${OUTROOT:-$GRAFT_REPO_ROOT/gpurun_out}/a18; mkdir -p $O
LIBS="base=fleet_amd/libfleetcodec.so ls1=ab/libls1.so ls2=ab/libls2.so" REPS=3 WORKLOADS="synth1m_256" STEPS=20 bash scripts/gpu_ab_multi.sh > $O/ladder_steps.txt 2>&1 || { tail -5 $O/ladder_steps.txt; exit 1; }
cat $O/ladder_steps.txt
OUT=$O/klibs LIBS="base=fleet_amd/libfleetcodec.so ls1=ab/libls1.so ls2=ab/libls2.so" WORKLOADS="synth1m_256" bash scripts/gpu_kardam_libs.sh || exit 1
