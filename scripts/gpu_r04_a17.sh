# r04 a17 (round-end tree): GPU suite, smoke, default bench, the N=2 same-device rehearsal (parity + approx blocks),
# then the r04 profile pass (kernel trace, FETCH/WRITE, SQ) of the headline and the extras
set -u
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=${OUTROOT:-$GRAFT_REPO_ROOT/gpurun_out}/a17; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1; rc=$?
tail -4 $O/tests.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 1
tail -1 $O/smoke.log
timeout -k 10 900 python3 bench.py > $O/bench.json 2> $O/bench.err || exit 1
python3 - $O/bench.json <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print("value", d["value"], "ms", d["ms_per_step"], "frac", d["roofline"]["frac"], "agg", d["roofline"].get("aggregation_alone", {}).get("frac"))
print({k: (v["pipelined"] or {}).get("ms_per_step") for k, v in d.get("extra", {}).items()})
print("approx", d.get("approx"))
PY
FLEET_BENCH_SAME_DEVICE=1 FLEET_BENCH_BACKEND=gloo timeout -k 10 600 python3 bench.py --gpus 2 --steps 4 --warmup 1 --no-cpu-baseline > $O/bench_n2.json 2> $O/bench_n2.err || { echo "n2 rc=$?"; tail -5 $O/bench_n2.err; exit 1; }
python3 - $O/bench_n2.json <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print("n2 value", d["value"], "parity", d.get("parity"), "strong parity", (d.get("strong") or {}).get("device", {}).get("parity"))
print("n2 approx", d.get("approx"))
PY
bash scripts/gpu_profile.sh r04f synth1m_256 cifar10_256 mnist64 cifar100_1024 || exit 1
