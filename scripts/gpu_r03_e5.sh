# final tree: the profile pass (kernel trace + FETCH/WRITE + SQ per workload) and the default bench line
set -u
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
bash scripts/gpu_profile.sh r03d synth1m_256 cifar10_256 mnist64 cifar100_1024 || exit 1
timeout -k 10 900 python bench.py > gpurun_out/r03d/bench_default.json 2> gpurun_out/r03d/bench_default.err; echo "bench rc=$?"
