# parity suite on the current build, then A/B of the variants
set -o pipefail
cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 180 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 600 python -u tools/ab_variants.py run --reps ${REPS:-3} > gpurun_out/ab.log 2>&1 || { echo "AB_FAIL"; tail -5 gpurun_out/ab.log; exit 1; }
grep SUMMARY gpurun_out/ab.log
