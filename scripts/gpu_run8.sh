set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python scripts/sweep_update.py mnist > gpurun_out/sweep_mnist.log 2>&1 && cat gpurun_out/sweep_mnist.log &&
timeout -k 10 300 python scripts/sweep_update.py cifar10 256 > gpurun_out/sweep_cifar.log 2>&1 && cat gpurun_out/sweep_cifar.log &&
timeout -k 10 300 python scripts/sweep_update.py synth1m 256 > gpurun_out/sweep_s1m.log 2>&1 && cat gpurun_out/sweep_s1m.log
