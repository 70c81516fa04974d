# prefetch distance of the stream update: configs[4] windows (update alone) and the headline step
set -u
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for L in base pf2 pf3; do FLEET_CODEC_LIB=$PWD/ab/lib_$L.so timeout -k 10 300 python -u scripts/strong_probe.py synth4m_4096 1,4,8 upd | sed "s/^/$L /" || exit 1; done
for L in base pf2 pf3; do FLEET_CODEC_LIB=$PWD/ab/lib_$L.so PROBE_M=1024 timeout -k 10 300 python -u scripts/strong_probe.py synth4m_4096 4 upd | sed "s/^/$L /" || exit 1; done
LIBS="base=ab/lib_base.so pf2=ab/lib_pf2.so pf3=ab/lib_pf3.so" REPS=2 WORKLOADS=synth1m_256 bash scripts/gpu_ab_multi.sh
