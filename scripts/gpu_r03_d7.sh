# client-chunked stream update: parity (chunk tests, fused step, full sizes, parity suite), then the strong-scaling windows
set -u
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_chunked.py tests/test_gpu_fused_step.py tests/test_gpu_parity.py tests/test_gpu_full_size.py > gpurun_out/d7_tests.log 2>&1; rc=$?; tail -3 gpurun_out/d7_tests.log; [ $rc = 0 ] || exit 1
for m in upd fused; do timeout -k 10 300 python -u scripts/strong_probe.py synth4m_4096 1,2,4,8 $m || exit 1; done
FLEET_UPDATE_CHUNK=0 timeout -k 10 300 python -u scripts/strong_probe.py synth4m_4096 1 fused || exit 1
