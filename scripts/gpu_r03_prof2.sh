# profile pass after the byte-table tiles (TAG r03b) + the Kardam plans (TAG r03k2)
set -u
bash scripts/gpu_profile.sh r03b synth1m_256 cifar10_256 mnist64 cifar100_1024 || exit 1
TAG=r03k2 bash scripts/gpu_kardam_plans.sh
