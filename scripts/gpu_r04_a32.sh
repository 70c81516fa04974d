# r04 a32: the fused-step tests on the tree (24 rows per encode block), then 48 rows (ab/librpb48.so)
# against 24, alternating on synth1m_256, and the default bench
set -u
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
O=${OUTROOT:-$GRAFT_REPO_ROOT/gpurun_out}/a32; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_fused_step.py tests/test_gpu_full_size.py tests/test_gpu_strong.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
LIBS="base=fleet_amd/libfleetcodec.so rpb48=ab/librpb48.so" REPS=3 WORKLOADS="synth1m_256" STEPS=20 bash scripts/gpu_ab_multi.sh > $O/rpb48.txt 2>&1 || { tail -5 $O/rpb48.txt; exit 1; }
cat $O/rpb48.txt
timeout -k 10 900 python3 bench.py > $O/bench.json 2> $O/bench.err || { tail -5 $O/bench.err; exit 1; }
python3 - $O/bench.json <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
r = d["roofline"]; a = r["aggregation_alone"]
print("value", d["value"], "ms", d["ms_per_step"], "frac", r["frac"], "agg", a["kernel_ms"], a["frac"])
PY
