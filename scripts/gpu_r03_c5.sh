set -u
timeout -k 10 300 python -u -m pytest -q --timeout 200 --timeout-method thread -m gpu tests/test_sampler_state.py tests/test_jni_shim.py tests/test_gpu_multi.py > gpurun_out/c5_tests.log 2>&1; echo "tests rc=$?"; tail -3 gpurun_out/c5_tests.log
EXTRA_TESTS= WORKLOADS="synth1m_256" bash scripts/gpu_ab_quick.sh > gpurun_out/c5_ab.log 2>&1; echo "ab rc=$?"; cat gpurun_out/c5_ab.log
FLEET_BENCH_SAME_DEVICE=1 FLEET_BENCH_BACKEND=gloo timeout -k 10 400 python bench.py --gpus 2 --steps 4 --warmup 1 --extras= --no-cpu-baseline --no-e2e --no-strong-block > gpurun_out/c5_rehearsal.json 2> gpurun_out/c5_rehearsal.err; echo "rehearsal rc=$?"; tail -c 1500 gpurun_out/c5_rehearsal.json; tail -5 gpurun_out/c5_rehearsal.err
