# CDF wave-kernel accumulation: CDF parity tests and probe timing.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1
O=gpurun_out/r04o
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_cdfdif.py -m gpu -v -p no:cacheprovider --timeout 200 --timeout-method thread > $O/pytest_cdf.log 2>&1 || { echo "PYTEST_FAIL rc=$?"; tail -5 $O/pytest_cdf.log; grep -E "^FAILED" $O/pytest_cdf.log | head; exit 1; }
tail -1 $O/pytest_cdf.log
for rep in 1 2 3; do
  timeout -k 10 120 python -u tools/cdf_probe.py --reps 20 > $O/cdf.$rep.log 2>&1 || { echo CDF_FAIL; exit 1; }
  cut -c1-140 $O/cdf.$rep.log
done
echo r04o-done
