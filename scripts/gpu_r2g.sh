set -u
O=gpurun_out/r2g; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -k "update" > $O/pytest.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -2 $O/pytest.log; [ $rc -ne 0 ] && exit 1
for MODE in tiled stream; do
 FLEET_UPDATE_MODE=$MODE timeout -k 10 300 python bench.py --workload cifar10_256 --extras= --no-cpu-baseline --no-e2e --steps 8 > $O/c_$MODE.json 2>&1; echo "$MODE rc=$? $(grep -o '"k_update_ms": [0-9.]*' $O/c_$MODE.json)"
done
FLEET_UPDATE_MODE=tiled FLEET_TILE_G=32 timeout -k 10 300 python bench.py --workload cifar10_256 --extras= --no-cpu-baseline --no-e2e --steps 8 > $O/c_t32.json 2>&1; echo "t32 rc=$? $(grep -o '"k_update_ms": [0-9.]*' $O/c_t32.json)"
FLEET_UPDATE_MODE=tiled FLEET_TILE_G=64 timeout -k 10 300 python bench.py --workload synth1m_256 --extras= --no-cpu-baseline --no-e2e --steps 8 > $O/s_t64.json 2>&1; echo "s_t64 rc=$? $(grep -o '"k_update_ms": [0-9.]*' $O/s_t64.json)"
