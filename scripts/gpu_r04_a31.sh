# r04 a31: rows per encode block of the fused stream step (6 / 24 against the tree's 12) now that
# the encode's waves run at priority 3, alternating on synth1m_256
set -u
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
O=${OUTROOT:-$GRAFT_REPO_ROOT/gpurun_out}/a31; mkdir -p $O
LIBS="base=fleet_amd/libfleetcodec.so rpb6=ab/librpb6.so rpb24=ab/librpb24.so" REPS=3 WORKLOADS="synth1m_256" STEPS=20 bash scripts/gpu_ab_multi.sh > $O/rpb.txt 2>&1 || { tail -5 $O/rpb.txt; exit 1; }
cat $O/rpb.txt
