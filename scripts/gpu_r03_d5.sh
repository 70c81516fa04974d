# strong-scaling per-rank windows of configs[4]: fused step vs its two kernels alone
set -u
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for m in upd enc fused; do timeout -k 10 300 python -u scripts/strong_probe.py synth4m_4096 1,4,8 $m || exit 1; done
timeout -k 10 300 python -u scripts/strong_probe.py synth1m_256 1,4,8 upd || exit 1
