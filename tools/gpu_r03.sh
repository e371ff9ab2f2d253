# GPU round script: parity tests, A/B of build variants, then the bench.
# Each GPU step under its own time limit; stop at the first failure.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
if [ "${SKIP_TESTS:-0}" != "1" ]; then
  timeout -k 10 600 python -u -m pytest ${TESTS:-tests} -m gpu -v -p no:cacheprovider --timeout 180 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?
  echo "pytest rc=$rc"; grep -E "FAILED|ERROR" gpurun_out/pytest_gpu.log | head -20; tail -2 gpurun_out/pytest_gpu.log
  # 1 = some tests failed (the run itself is sound): go on to the timings
  [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
fi
if [ "${SKIP_AB:-0}" != "1" ]; then
  timeout -k 10 900 python -u tools/ab_variants.py run --reps ${REPS:-3} ${NAMES:+--names $NAMES} > gpurun_out/ab.log 2>&1 || { echo "AB_FAIL rc=$?"; tail -5 gpurun_out/ab.log; exit 1; }
  grep SUMMARY gpurun_out/ab.log
fi
timeout -k 10 400 python -u bench.py --steps 20 --warmup 3 --cpu-seconds 5 > gpurun_out/bench.log 2>&1 || { echo "BENCH_FAIL rc=$?"; tail -5 gpurun_out/bench.log; exit 1; }
tail -1 gpurun_out/bench.log
