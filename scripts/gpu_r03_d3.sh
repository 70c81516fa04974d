# fused-step launch knobs on the tree's library: encode-wave priority x plain/balanced update grid, rows per encode block
set -u
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
L=fleet_amd/libfleetcodec.so
LIBS="base=$L prio1=$L,FLEET_FUSED_ENC_PRIO=1 mixed=$L,FLEET_FUSED_PLAIN=0 mixp1=$L,FLEET_FUSED_PLAIN=0,FLEET_FUSED_ENC_PRIO=1 mixp2=$L,FLEET_FUSED_PLAIN=0,FLEET_FUSED_ENC_PRIO=2 rpb24=$L,FLEET_FUSED_RPB=24 rpb6=$L,FLEET_FUSED_RPB=6" REPS=2 WORKLOADS=synth1m_256 bash scripts/gpu_ab_multi.sh
