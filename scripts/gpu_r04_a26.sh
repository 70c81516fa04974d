# r04 a26: the fused step's update waves laddered from priority 2 (ab/liflt2.so: 2, 1, 0, 0; the
# encode's waves at 3 above them all) against the tree's 3 -> 0, alternating on synth1m_256
set -u
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
O=${OUTROOT:-$GRAFT_REPO_ROOT/gpurun_out}/a26; mkdir -p $O
LIBS="base=fleet_amd/libfleetcodec.so lt2=ab/liflt2.so" REPS=3 WORKLOADS="synth1m_256" STEPS=20 bash scripts/gpu_ab_multi.sh > $O/fused_ladder_top.txt 2>&1 || { tail -5 $O/fused_ladder_top.txt; exit 1; }
cat $O/fused_ladder_top.txt
