# issue priority of the balanced grid's value-per-lane waves: headline (update alone) and configs[4]'s N=4 window
set -u
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for L in base s1p1 s1p2; do FLEET_CODEC_LIB=$PWD/ab/lib_$L.so PROBE_M=1024 timeout -k 10 300 python -u scripts/strong_probe.py synth4m_4096 4 upd | sed "s/^/$L /" || exit 1; done
for L in base s1p1 s1p2; do FLEET_CODEC_LIB=$PWD/ab/lib_$L.so timeout -k 10 300 python -u scripts/strong_probe.py synth4m_4096 1 upd | sed "s/^/$L /" || exit 1; done
LIBS="base=ab/lib_base.so s1p1=ab/lib_s1p1.so s1p2=ab/lib_s1p2.so" REPS=2 WORKLOADS=synth1m_256 bash scripts/gpu_ab_multi.sh
