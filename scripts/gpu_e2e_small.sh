set -u
O=gpurun_out/e2e_small; mkdir -p $O
for T in 1 3 8; do echo "T=$T"; FLEET_STAGE_THREADS=$T timeout -k 10 200 python scripts/probe_e2e_small.py mnist64 cifar10_256 || exit 1; done
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 200 rocprofv3 --kernel-trace --memory-copy-trace --stats -d $O/prof -o run -- python scripts/probe_e2e_small.py mnist64 > $O/prof.log 2>&1 || exit 1
