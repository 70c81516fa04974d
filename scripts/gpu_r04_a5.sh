# r04 a5: A/B of the issue-priority ladder in the stream kernels (ab/libladder.so, FLEET_PRIO_LADDER=1)
# against the tree's library, alternating on one box
set -u
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
LIBS="base=fleet_amd/libfleetcodec.so ladder=ab/libladder.so" REPS=3 WORKLOADS="synth1m_256" STEPS=20 bash scripts/gpu_ab_multi.sh || exit 1
LIBS="base=fleet_amd/libfleetcodec.so ladder=ab/libladder.so" REPS=1 WORKLOADS="synth4m_4096" STEPS=4 bash scripts/gpu_ab_multi.sh || exit 1
# MNIST-64 pipelined tiles: phase timestamps (scripts/ubench_tiled.hip, FLEET_TIMING build)
timeout -k 10 120 ./scripts/ubench_tiled || exit 1
