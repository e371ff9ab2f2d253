# Per-call level-0 constants: summing-path parity (bitwise sequences), A/B.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1
O=gpurun_out/r04p
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests -m gpu -v -p no:cacheprovider --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo "PYTEST_FAIL rc=$?"; tail -5 $O/pytest_gpu.log; grep -E "^FAILED" $O/pytest_gpu.log | head; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 600 python -u tools/ab_variants.py run --reps 3 --names default,l0off > $O/ab.log 2>&1 || { echo AB_FAIL; tail -5 $O/ab.log; exit 1; }
grep -v SUMMARY $O/ab.log | cut -c1-200
grep SUMMARY $O/ab.log
echo r04p-done
