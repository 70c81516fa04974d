# r04 a6: Kardam's pipelined form (producers store p, k_kardam_finish) and in-place G rows; the
# Kardam A/B per workload (HEAD-of-a5 library: k_update<1, true> / NW=8 pipe + reduce; the tree;
# the tree's stream form on the plain grid); the issue-priority ladder A/B; MNIST-64 phase stamps
set -u
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
O=${OUTROOT:-$GRAFT_REPO_ROOT/gpurun_out}/a6; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_kardam_fused.py tests/test_gpu_parity.py tests/test_gpu_fused_step.py -m gpu -x -q --timeout 200 --timeout-method thread -k "kardam or keep_slots or under_plans or stream" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
OUT=$O/klibs LIBS="head=ab/libhead.so tree=fleet_amd/libfleetcodec.so plain=fleet_amd/libfleetcodec.so,FLEET_EXPERIMENTS=grid=plain" WORKLOADS="synth1m_256" bash scripts/gpu_kardam_libs.sh || exit 1
OUT=$O/klibs LIBS="head=ab/libhead.so tree=fleet_amd/libfleetcodec.so" WORKLOADS="mnist64 cifar10_256" bash scripts/gpu_kardam_libs.sh || exit 1
LIBS="base=fleet_amd/libfleetcodec.so ladder=ab/libladder.so" REPS=3 WORKLOADS="synth1m_256" STEPS=20 bash scripts/gpu_ab_multi.sh > $O/ladder.txt 2>&1 || { tail -5 $O/ladder.txt; exit 1; }
cat $O/ladder.txt
timeout -k 10 120 ./scripts/ubench_tiled > $O/ubench_tiled.log 2>&1 || exit 1
tail -20 $O/ubench_tiled.log
