set -u
O=gpurun_out/r2k; mkdir -p $O
timeout -k 10 120 ./scripts/ubench_tiled > $O/ubench_tiled.txt 2>&1; echo "ubench rc=$?"; grep "wp0 TG=16.*M=64" $O/ubench_tiled.txt
bash scripts/gpu_r2j.sh
