# per-rank local step of the strong-scaling value at N = 1..8 (rank 0's window, one GPU)
set -u
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u scripts/strong_probe.py synth1m_256 1,2,3,4,6,8 || exit 1
timeout -k 10 400 python -u scripts/strong_probe.py synth4m_4096 1,2,4,8 || exit 1
