# Kardam plans after the one-wave reduce: GPU Kardam tests, then per-kernel stats per
# workload, mnist64 also with the 5-wave pipe (FLEET_KARDAM_PIPE_NW=5)
set -u
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kardam_fused.py tests/test_updater.py -m gpu > gpurun_out/c11_tests.log 2>&1; rc=$?; tail -2 gpurun_out/c11_tests.log; [ $rc = 0 ] || exit 1
TAG=c11 bash scripts/gpu_kardam_plans.sh || exit 1
FLEET_KARDAM_PIPE_NW=5 TAG=c11nw5 WORKLOADS=mnist64 bash scripts/gpu_kardam_plans.sh || exit 1
