# final tree: Kardam's side outputs on every launch plan (kernel stats per workload)
set -u
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_kardam_fused.py > gpurun_out/e6_tests.log 2>&1; rc=$?; tail -1 gpurun_out/e6_tests.log; [ $rc = 0 ] || exit 1
TAG=r03kf bash scripts/gpu_kardam_plans.sh || exit 1
