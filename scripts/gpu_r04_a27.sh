# r04 a27: with the ladder in place, the stream aggregation's SIMD-balanced grid (the default) against
# the plain grid and the value-per-lane grid (plan overrides), alternating on synth1m_256 / synth4m_4096
set -u
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
O=${OUTROOT:-$GRAFT_REPO_ROOT/gpurun_out}/a27; mkdir -p $O
LIBS="auto=fleet_amd/libfleetcodec.so plain=fleet_amd/libfleetcodec.so,FLEET_EXPERIMENTS=grid=plain" REPS=3 WORKLOADS="synth1m_256" STEPS=20 bash scripts/gpu_ab_multi.sh > $O/grid.txt 2>&1 || { tail -5 $O/grid.txt; exit 1; }
LIBS="auto=fleet_amd/libfleetcodec.so plain=fleet_amd/libfleetcodec.so,FLEET_EXPERIMENTS=grid=plain" REPS=1 WORKLOADS="synth4m_4096" STEPS=4 bash scripts/gpu_ab_multi.sh >> $O/grid.txt 2>&1 || { tail -5 $O/grid.txt; exit 1; }
cat $O/grid.txt
