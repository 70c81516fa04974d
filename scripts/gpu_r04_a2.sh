# r04 a2: header slots out of the chain (keep_bits) -- GPU suite, then configs[4]'s
# strong-scaling windows before (ab/libprev.so) and after
set -u
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/a2; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1; rc=$?
tail -5 $O/tests.log
[ $rc -eq 0 ] || exit 1
PROBE_M=1024 FLEET_CODEC_LIB=ab/libprev.so timeout -k 10 300 python3 scripts/strong_probe.py synth4m_4096 4,8 upd > $O/probe.log 2>&1 || exit 1
PROBE_M=1024 timeout -k 10 300 python3 scripts/strong_probe.py synth4m_4096 4,8 upd >> $O/probe.log 2>&1 || exit 1
timeout -k 10 600 python3 scripts/strong_probe.py synth4m_4096 1,4,8 fused >> $O/probe.log 2>&1 || exit 1
cat $O/probe.log
