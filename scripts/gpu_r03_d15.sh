# MNIST-64 pipelined step: the encode's blocks first or last in k_update_pipe's grid, rows per encode block
set -u
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_fused_step.py > gpurun_out/d15_tests.log 2>&1; rc=$?; tail -1 gpurun_out/d15_tests.log; [ $rc = 0 ] || exit 1
L=fleet_amd/libfleetcodec.so
LIBS="last=$L first=$L,FLEET_PIPE_ENC_FIRST=1 last_rpb4=$L,FLEET_ENCODE_RPB=4 first_rpb4=$L,FLEET_PIPE_ENC_FIRST=1,FLEET_ENCODE_RPB=4 first_rpb16=$L,FLEET_PIPE_ENC_FIRST=1,FLEET_ENCODE_RPB=16" REPS=3 WORKLOADS=mnist64 STEPS=200 bash scripts/gpu_ab_multi.sh
