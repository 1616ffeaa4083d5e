set -o pipefail
out=gpurun_out/r05_lead; mkdir -p $out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $out/pytest.log 2>&1 || { echo "pytest failed rc=$?"; tail -30 $out/pytest.log; exit 1; }
tail -1 $out/pytest.log
bash tools/ab_lib.sh run $out/ab 3 --steps 300 --no-cpu-baseline --spread-steps 0 --replay-steps 0 --no-nodedup --cutoff-steps 0
