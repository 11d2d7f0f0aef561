set -u
mkdir -p gpurun_out
rm -f gpurun_out/ab_quick.txt
bash scripts/ab_quick.sh 3 || exit 1
bash scripts/ab_quick.sh 3 --launch per-frame || exit 1
bash scripts/ab_quick.sh 2 --scene bunny || exit 1
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread > gpurun_out/pytest_ring.log 2>&1
echo "tests rc=$?"; tail -1 gpurun_out/pytest_ring.log
