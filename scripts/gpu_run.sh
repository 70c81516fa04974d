# Parameterised GPU call: run named steps in order, each under its own time limit,
# stopping at the first failure. Output under gpurun_out/$TAG/.
# usage (through gpurun, from the repo root):
#   bash scripts/gpu_run.sh tag=r05b0 tests smoke bench strong windows:cifar10_256 profile
#   (tag=NAME first, or TAG in the environment: the output directory)
# steps:
#   tests            full pytest -m gpu
#   smoke            __graft_entry__.smoke()
#   bench            the default bench line (bench_default.json)
#   sqlds:W:N:MODE   LDS counters (bank conflicts, unaligned stalls) of strong_probe W at N, MODE
#   bin:PATH         a prebuilt dev binary
#   klibs:W1,W2      Kardam vs plain per library build in LIBS (scripts/gpu_kardam_libs.sh)
#   benchn:N         bench.py --gpus N with every rank on device 0 over gloo (the N-rank path rehearsed)
#   strong[:W]       per-rank pipelined windows of W (default synth1m_256) at N = 1, 2, 4, 8
#                    on one GPU (scripts/strong_probe.py), fused / update-only
#   windows:W        W at N = 1 only: the fused step, the update alone, the encode alone
#   profile[:W,..]   scripts/gpu_profile.sh $TAG (kernel trace + PMC passes)
#   ab               scripts/gpu_ab_multi.sh (LIBS, WORKLOADS, REPS from the environment)
#   kardam[:W,..]    Kardam side outputs vs the plain update (scripts/kardam_ab.py under rocprofv3)
#   py:FILE          python3 FILE (a probe script), output in $TAG/FILE.log
#   pyargs:FILE|A|B  python3 FILE A B (arguments split at '|'), appended to $TAG/FILE.log
#   pytest:EXPR      pytest -m gpu -k EXPR (a subset), output in $TAG/pytest.log
#   sq:W:N:MODE      SQ counters (8) + GRBM_GUI_ACTIVE + kernel trace of strong_probe.py W N MODE
#                    (rank 0's window at N ranks; MODE fused | upd | enc), per-kernel summary
#   sqk:W            the same counters over scripts/kardam_ab.py W (Kardam forms and the plain update)
#   trace:W:N:MODE   per-wave phase trace of the tile kernels (scripts/tile_trace.py; needs
#                    FLEET_CODEC_LIB=ab/trace.so, a FLEET_TRACE build)
#   plans:W:N:MODE:P1|P2|..  same-process A/B of launch plans (scripts/plan_ab.py; '-' = default,
#                    ';' between a plan's keys)
#   env:VAR=VALUE    export VAR for the steps after it (env:VAR= unsets it), e.g.
#                    'env:FLEET_EXPERIMENTS=update=tiled;tile=weave6' (quote the ';')
set -u -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$PWD}"
TAG=${TAG:-run}
case ${1:-} in tag=*) TAG=${1#tag=}; shift ;; esac
O=${OUTROOT:-$PWD/gpurun_out}/$TAG; mkdir -p "$O"
for step in "$@"; do
  name=${step%%:*}; arg=""; [ "$name" != "$step" ] && arg=${step#*:}
  echo "== $step"
  case $name in
    tests)
      timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$O/tests.log" 2>&1 \
        || { tail -30 "$O/tests.log"; exit 1; }
      tail -1 "$O/tests.log" ;;
    smoke)
      timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.log" 2>&1 || { tail -20 "$O/smoke.log"; exit 1; }
      tail -1 "$O/smoke.log" ;;
    bench)
      timeout -k 10 900 python3 bench.py > "$O/bench_default.json" 2> "$O/bench_default.err" || { tail -20 "$O/bench_default.err"; exit 1; }
      cut -c1-400 "$O/bench_default.json" ;;
    benchn)
      # the N-rank bench path rehearsed on one GPU: N ranks on device 0, gloo collectives
      # (a readiness check, its times measure nothing)
      FLEET_BENCH_SAME_DEVICE=1 FLEET_BENCH_BACKEND=gloo timeout -k 10 1200 python3 bench.py --gpus "$arg" --steps 8 \
        --warmup 2 > "$O/bench_n${arg}_same_device.json" 2> "$O/bench_n${arg}_same_device.err" \
        || { tail -20 "$O/bench_n${arg}_same_device.err"; exit 1; }
      cut -c1-300 "$O/bench_n${arg}_same_device.json" ;;
    strong)
      W=${arg:-synth1m_256}
      for mode in fused upd; do
        timeout -k 10 300 python3 scripts/strong_probe.py "$W" 1,2,4,8 $mode >> "$O/strong_$W.txt" 2>&1 || { tail -20 "$O/strong_$W.txt"; exit 1; }
      done
      cat "$O/strong_$W.txt" ;;
    windows)
      for mode in fused upd enc; do
        timeout -k 10 300 python3 scripts/strong_probe.py "$arg" 1 $mode >> "$O/windows_$arg.txt" 2>&1 || { tail -20 "$O/windows_$arg.txt"; exit 1; }
      done
      cat "$O/windows_$arg.txt" ;;
    profile)
      OUTROOT=$(dirname "$O") bash scripts/gpu_profile.sh "$TAG" ${arg//,/ } || exit 1 ;;
    ab)
      bash scripts/gpu_ab_multi.sh > "$O/ab.txt" 2>&1 || { tail -20 "$O/ab.txt"; exit 1; }
      cat "$O/ab.txt" ;;
    kardam)
      for W in ${arg:-mnist64 cifar10_256 synth1m_256}; do
        W=${W//,/ }
        for w in $W; do
          timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/kardam_$w" -o run -- \
            python3 scripts/kardam_ab.py "$w" > "$O/kardam_$w.log" 2>&1 || { tail -20 "$O/kardam_$w.log"; exit 1; }
          echo "-- $w"
          python3 -c "
import csv
for r in csv.DictReader(open('$O/kardam_$w/run_kernel_stats.csv')):
    n = r['Name']
    if 'k_update' in n or 'k_kardam' in n:
        print('%-42s calls %4s avg %8.1f us' % (n.split('(')[0].replace('void fleet::', '').replace('fleet::', ''),
                                                r['Calls'], float(r['AverageNs']) / 1e3))
" | tee -a "$O/kardam.txt"
        done
      done ;;
    env)
      v=${arg%%=*}
      if [ -z "${arg#*=}" ]; then unset "$v"; else export "$arg"; fi
      echo "$v=${!v:-}" ;;
    pytest)
      timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "$arg" \
        >> "$O/pytest.log" 2>&1 || { tail -30 "$O/pytest.log"; exit 1; }
      tail -1 "$O/pytest.log" ;;
    sq)
      IFS=: read -r W N MODE <<< "$arg"
      D="$O/sq_${W}_n${N}_${MODE}${SQTAG:-}"
      timeout -s KILL 240 rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_BUSY_CU_CYCLES SQ_WAVE_CYCLES \
        SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE --output-format csv -d "$D" -o run \
        -- python3 scripts/strong_probe.py "$W" "$N" "$MODE" > "$D.log" 2>&1 || { tail -20 "$D.log"; exit 1; }
      EC=$(python3 -c "import sys; sys.path.insert(0,'.'); import bench; from fleet_amd.layouts import LAYOUTS; l,m,_=bench.WORKLOADS['$W']; print(m*LAYOUTS[l].n_up/$N)")
      echo "-- $W N=$N $MODE ${FLEET_EXPERIMENTS:-default}" | tee -a "$O/sq.txt"
      python3 scripts/pmc_kernels.py "$D" "$EC" | grep -E "k_update|k_encode" | tee -a "$O/sq.txt" ;;
    sqlds)
      # LDS pass: bank conflicts / unaligned stalls / LDS-array cycles per kernel
      IFS=: read -r W N MODE <<< "$arg"
      D="$O/sqlds_${W}_n${N}_${MODE}${SQTAG:-}"
      timeout -s KILL 240 rocprofv3 --kernel-trace --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE \
        SQ_LDS_UNALIGNED_STALL SQ_LDS_ADDR_CONFLICT SQ_WAVES SQ_INSTS_VALU SQ_BUSY_CU_CYCLES --output-format csv -d "$D" \
        -o run -- python3 scripts/strong_probe.py "$W" "$N" "$MODE" > "$D.log" 2>&1 || { tail -20 "$D.log"; exit 1; }
      echo "-- lds $W N=$N $MODE ${SQTAG:-} ${FLEET_EXPERIMENTS:-default}" | tee -a "$O/sqlds.txt"
      python3 scripts/pmc_kernels.py "$D" | grep -E "k_update|k_encode" | tee -a "$O/sqlds.txt" ;;
    sqk)
      W=$arg
      D="$O/sqk_${W}${SQTAG:-}"
      timeout -s KILL 240 rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_BUSY_CU_CYCLES SQ_WAVE_CYCLES \
        SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE --output-format csv -d "$D" -o run \
        -- python3 scripts/kardam_ab.py "$W" > "$D.log" 2>&1 || { tail -20 "$D.log"; exit 1; }
      EC=$(python3 -c "import sys; sys.path.insert(0,'.'); import bench; from fleet_amd.layouts import LAYOUTS; l,m,_=bench.WORKLOADS['$W']; print(m*LAYOUTS[l].n_up)")
      echo "-- kardam $W ${FLEET_EXPERIMENTS:-default}" | tee -a "$O/sq.txt"
      python3 scripts/pmc_kernels.py "$D" "$EC" | grep -E "k_update|k_kardam" | tee -a "$O/sq.txt" ;;
    trace)
      IFS=: read -r W N MODE <<< "$arg"
      echo "-- ${FLEET_EXPERIMENTS:-default}" >> "$O/trace.txt"
      PL=$(echo "${FLEET_EXPERIMENTS:-default}" | tr ';=,' '___')
      TRACE_OUT="$O/bt_${W}_n${N}_${MODE}_${PL}.npy" timeout -k 10 300 python3 scripts/tile_trace.py "$W" "$N" "$MODE" \
        >> "$O/trace.txt" 2>&1 || { tail -20 "$O/trace.txt"; exit 1; }
      tail -14 "$O/trace.txt" ;;
    plans)
      IFS=: read -r W N MODE PL <<< "$arg"
      IFS='|' read -r -a PA <<< "$PL"
      timeout -k 10 600 python3 scripts/plan_ab.py "$W" "$N" "$MODE" "${PA[@]}" 2>&1 | grep -v amdgpu.ids >> "$O/plans.txt" \
        || { tail -20 "$O/plans.txt"; exit 1; }
      tail -$((${#PA[@]} + 1)) "$O/plans.txt" ;;
    pyargs)
      IFS='|' read -r -a PA <<< "$arg"
      timeout -k 10 600 python3 "${PA[@]}" 2>&1 | grep -v amdgpu.ids >> "$O/$(basename "${PA[0]}").log" \
        || { tail -30 "$O/$(basename "${PA[0]}").log"; exit 1; }
      tail -12 "$O/$(basename "${PA[0]}").log" ;;
    bin)
      # a prebuilt dev binary (e.g. ab6/ubench_valu2): its output to bin_<name>.log
      timeout -k 10 300 "$arg" > "$O/bin_$(basename "$arg").log" 2>&1 || { tail -30 "$O/bin_$(basename "$arg").log"; exit 1; }
      tail -40 "$O/bin_$(basename "$arg").log" ;;
    klibs)
      # Kardam per library build (LIBS) on the workloads in arg (comma-separated)
      OUT="$O/klibs" WORKLOADS="${arg//,/ }" bash scripts/gpu_kardam_libs.sh > "$O/klibs.txt" 2>&1 || { tail -20 "$O/klibs.txt"; exit 1; }
      cat "$O/klibs.txt" ;;
    py)
      timeout -k 10 600 python3 "$arg" > "$O/$(basename "$arg").log" 2>&1 || { tail -30 "$O/$(basename "$arg").log"; exit 1; }
      tail -40 "$O/$(basename "$arg").log" ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
echo "== done"
