# r04 a15: the ladder in the fused step's update waves (ab/libfl*.so: encode waves at priority
# 0 / 1 / 2) against the tree, alternating on synth1m_256; the Kardam tests and per-workload
# numbers of the tree (the ladder now in the Kardam stream form too)
set -u
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
O=${OUTROOT:-$GRAFT_REPO_ROOT/gpurun_out}/a15; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_kardam_fused.py tests/test_gpu_parity.py tests/test_gpu_fused_step.py -m gpu -x -q --timeout 200 --timeout-method thread -k "kardam or keep_slots or stream or under_plans" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
LIBS="base=fleet_amd/libfleetcodec.so fl=ab/libfl.so fl1=ab/libfl1.so fl2=ab/libfl2.so" REPS=3 WORKLOADS="synth1m_256" STEPS=20 bash scripts/gpu_ab_multi.sh > $O/fused_ladder.txt 2>&1 || { tail -5 $O/fused_ladder.txt; exit 1; }
cat $O/fused_ladder.txt
OUT=$O/klibs LIBS="tree=fleet_amd/libfleetcodec.so" WORKLOADS="mnist64 cifar10_256 synth1m_256" bash scripts/gpu_kardam_libs.sh || exit 1
