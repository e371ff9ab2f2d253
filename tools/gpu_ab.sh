# GPU: parity tests, then A/B of build variants, then the bench. No retries.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -m gpu -v -p no:cacheprovider --timeout 240 > gpurun_out/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 900 python tools/ab_variants.py run --reps ${REPS:-3} > gpurun_out/ab.log 2>&1 || { echo "AB_FAIL rc=$?"; tail -5 gpurun_out/ab.log; exit 1; }
grep SUMMARY gpurun_out/ab.log
timeout -k 10 400 python bench.py --steps 20 --warmup 3 --cpu-seconds 5 > gpurun_out/bench.log 2>&1 || { echo "BENCH_FAIL rc=$?"; exit 1; }
tail -1 gpurun_out/bench.log
