# Kardam with 12-byte prev / G row accesses: Kardam tests, plan stats
set -u
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kardam_fused.py tests/test_updater.py -m gpu > gpurun_out/c19_tests.log 2>&1; rc=$?; tail -2 gpurun_out/c19_tests.log; [ $rc = 0 ] || exit 1
TAG=c19 bash scripts/gpu_kardam_plans.sh
