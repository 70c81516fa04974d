# r04 a11: the tree's check first (full GPU suite, smoke, default bench), then the Kardam A/B
# (a5 HEAD library against the tree, alternating) and the tile-ladder A/B
set -u
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
O=${OUTROOT:-$GRAFT_REPO_ROOT/gpurun_out}/a11; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 1
tail -1 $O/smoke.log
timeout -k 10 900 python3 bench.py > $O/bench.json 2> $O/bench.err || { tail -5 $O/bench.err; exit 1; }
python3 - $O/bench.json <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
r = d["roofline"]; a = r["aggregation_alone"]
print("value", d["value"], "frac", r["frac"], "agg", a["kernel"], a["kernel_ms"], a["frac"], "approx", (d.get("approx") or {}).get("equals_exact_bytes"))
PY
for r in 1 2; do
  OUT=$O/klibs$r LIBS="head=ab/libhead.so tree=fleet_amd/libfleetcodec.so" WORKLOADS="mnist64 synth1m_256 cifar10_256" bash scripts/gpu_kardam_libs.sh || exit 1
done
LIBS="base=fleet_amd/libfleetcodec.so tladder=ab/libtladder.so" REPS=3 WORKLOADS="cifar10_256 cifar100_1024" STEPS=20 bash scripts/gpu_ab_multi.sh > $O/tile_ladder.txt 2>&1 || { tail -5 $O/tile_ladder.txt; exit 1; }
cat $O/tile_ladder.txt
