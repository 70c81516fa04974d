# r04 a3: the launch-plan refactor (validated plan overrides, dropped variants) -- GPU suite, smoke, default bench
set -u
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=${OUTROOT:-$GRAFT_REPO_ROOT/gpurun_out}/a3; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1; rc=$?
tail -15 $O/tests.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 1
tail -2 $O/smoke.log
timeout -k 10 600 python3 bench.py > $O/bench.json 2> $O/bench.err || exit 1
python3 -c "
import json; d=json.loads(open('$O/bench.json').read().strip().splitlines()[-1])
print(d['value'], d['ms_per_step'], d['roofline']['frac'], d['roofline'].get('aggregation_alone',{}).get('frac'))
print({k: (v.get('pipelined',{}).get('ms_per_step'), v.get('ms_per_step')) for k, v in d.get('extra',{}).items()})
print(d.get('strong'))
"
