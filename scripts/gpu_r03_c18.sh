# stream Kardam kernel with DPP wave sums in the ILP unit: Kardam tests, plan stats; then the narrow-tile width A/B
set -u
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kardam_fused.py tests/test_updater.py -m gpu > gpurun_out/c18_tests.log 2>&1; rc=$?; tail -2 gpurun_out/c18_tests.log; [ $rc = 0 ] || exit 1
TAG=c18 WORKLOADS="synth1m_256 cifar10_256" bash scripts/gpu_kardam_plans.sh || exit 1
bash scripts/gpu_r03_c17.sh
