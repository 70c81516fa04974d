# the update alone on configs[4]'s N=4 window: client count, grid form
set -u
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for m in 256 1024 2048 4096; do PROBE_M=$m timeout -k 10 300 python -u scripts/strong_probe.py synth4m_4096 4 upd || exit 1; done
FLEET_UPDATE_MIXED=0 timeout -k 10 300 python -u scripts/strong_probe.py synth4m_4096 4 upd || exit 1
PROBE_M=1024 timeout -k 10 300 python -u scripts/strong_probe.py synth4m_4096 1 upd || exit 1
