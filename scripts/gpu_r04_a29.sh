# r04 a29: round-end tree: the whole GPU suite, smoke, the default bench, Kardam per workload
set -u
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
O=${OUTROOT:-$GRAFT_REPO_ROOT/gpurun_out}/a29; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 1
tail -1 $O/smoke.log
timeout -k 10 900 python3 bench.py > $O/bench.json 2> $O/bench.err || { tail -5 $O/bench.err; exit 1; }
python3 - $O/bench.json <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
r = d["roofline"]; a = r["aggregation_alone"]
print("value", d["value"], "ms", d["ms_per_step"], "frac", r["frac"], "agg", a["kernel_ms"], a["frac"])
PY
OUT=$O/klibs LIBS="tree=fleet_amd/libfleetcodec.so" WORKLOADS="mnist64 cifar10_256 synth1m_256" bash scripts/gpu_kardam_libs.sh || exit 1
