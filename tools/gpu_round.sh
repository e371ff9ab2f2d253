# One gpurun call: GPU tests, bench, stress probe, kernel trace of both.
# Every GPU step has its own time limit; the first failure ends the script.
#   gpurun --timeout 1100 -- 'bash tools/gpu_round.sh'
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/round
mkdir -p $OUT
STAGE=${STAGE:-all}
if [ "$STAGE" = all ] || [ "$STAGE" = tests ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 150 --timeout-method thread \
    > $OUT/pytest_gpu.log 2>&1 || { echo "TESTS_FAIL rc=$?"; tail -30 $OUT/pytest_gpu.log; exit 1; }
  tail -3 $OUT/pytest_gpu.log
fi
if [ "$STAGE" = all ] || [ "$STAGE" = bench ]; then
  timeout -k 10 300 python bench.py > $OUT/bench.log 2>&1 || { echo "BENCH_FAIL rc=$?"; tail -20 $OUT/bench.log; exit 1; }
  tail -1 $OUT/bench.log
  timeout -k 10 300 python tools/stress_probe.py > $OUT/stress.log 2>&1 || { echo "STRESS_FAIL rc=$?"; tail -20 $OUT/stress.log; exit 1; }
  cat $OUT/stress.log
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace_stress -o t -- python3 tools/stress_probe.py --reps 5 > $OUT/trace_stress.log 2>&1 || { echo "TRACE_FAIL rc=$?"; exit 1; }
  echo trace-ok
fi
