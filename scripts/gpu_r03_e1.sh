# round-3 refresh after the stage-C offset change: full GPU suite + smoke + default bench, then a profile pass
set -u
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
bash scripts/gpu_final.sh || exit 1
grep -c '^{' gpurun_out/final/bench_default.json
bash scripts/gpu_profile.sh r03c synth1m_256 cifar10_256 mnist64 cifar100_1024 || exit 1
