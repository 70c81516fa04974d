# full GPU test suite, profile pass (traces + PMC) and the default bench line
# usage: bash scripts/gpu_refresh.sh [TAG]   (writes gpurun_out/TAG; scripts/sync_profiles.sh TAG copies it)
set -u
TAG=${1:-r02}
O=gpurun_out/$TAG; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -2 $O/pytest.log; [ $rc -ne 0 ] && exit 1
bash scripts/gpu_profile.sh $TAG || exit 1
timeout -k 10 900 python bench.py > $O/bench_default.json 2> $O/bench_default.err; echo "bench rc=$?"; tail -c 600 $O/bench_default.json
