# r04 a7: k_kardam_finish with the header list in LDS and two groups per lane, the Kardam stream
# form on the plain grid, the issue-priority ladder in the standalone stream kernel: GPU tests of
# those paths, the Kardam A/B against the a5 HEAD library, and the default bench
set -u
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
O=${OUTROOT:-$GRAFT_REPO_ROOT/gpurun_out}/a7; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_kardam_fused.py tests/test_gpu_parity.py tests/test_gpu_fused_step.py tests/test_gpu_strong.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
OUT=$O/klibs LIBS="head=ab/libhead.so tree=fleet_amd/libfleetcodec.so" WORKLOADS="mnist64 synth1m_256" bash scripts/gpu_kardam_libs.sh || exit 1
timeout -k 10 900 python3 bench.py > $O/bench.json 2> $O/bench.err || { tail -5 $O/bench.err; exit 1; }
python3 - $O/bench.json <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
r = d["roofline"]; a = r["aggregation_alone"]
print("value", d["value"], "frac", r["frac"], "agg", a["kernel"], a["kernel_ms"], a["frac"])
print({k: (v.get("update_kernel"), v.get("update_kernel_ms"), (v["pipelined"] or {}).get("ms_per_step")) for k, v in d.get("extra", {}).items()})
PY
