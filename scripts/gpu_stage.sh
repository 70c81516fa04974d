# ingress staging (f3): GPU tests, then host-path timing by H2D pieces
set -u
O=gpurun_out/stage; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -2 $O/pytest.log; [ $rc -ne 0 ] && exit 1
for P in 1 3; do
  FLEET_STAGE_PIECES=$P timeout -k 10 120 python scripts/probe_e2e2.py > $O/probe_$P.txt 2>&1 || exit 1
  echo "pieces $P: $(tail -1 $O/probe_$P.txt)"
done
