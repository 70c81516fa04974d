# configs[4]'s N=4 window, update alone at M = 1024: upload rows as wide as the window (5.6 MB) or 2x / 4x wider
set -u
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for pm in 1 2 4; do PROBE_M=1024 PROBE_PITCH_MULT=$pm timeout -k 10 300 python -u scripts/strong_probe.py synth4m_4096 4 upd || exit 1; done
PROBE_M=256 PROBE_PITCH_MULT=4 timeout -k 10 300 python -u scripts/strong_probe.py synth4m_4096 4 upd || exit 1
