# baseline of this session: GPU parity tests, default bench, K variants of the stream kernel
set -u
O=gpurun_out/r2a; mkdir -p $O
fatal() { rc=$1; if [ $rc -ge 124 ]; then echo "fatal rc=$rc ($2)"; exit $rc; fi; }
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -5 $O/pytest_gpu.log; fatal $rc pytest
timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err; rc=$?; echo "bench rc=$rc"; fatal $rc bench
for K in 1 2 4; do
  FLEET_UPDATE_K=$K timeout -k 10 200 python bench.py --workload synth1m_256 --extras= --no-cpu-baseline --no-e2e --steps 10 > $O/k$K.json 2>&1; rc=$?
  echo "K=$K rc=$rc $(grep -o '"k_update_ms": [0-9.]*' $O/k$K.json)"; fatal $rc k$K
done
