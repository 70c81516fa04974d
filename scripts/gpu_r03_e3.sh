# the cleaned tree: full GPU suite + smoke + default bench, then the strong windows
set -u
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
bash scripts/gpu_final.sh || exit 1
timeout -k 10 300 python -u scripts/strong_probe.py synth1m_256 1,2,4,8 fused || exit 1
