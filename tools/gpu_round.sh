# One gpurun call: GPU tests, smoke, bench (headline + stress field).
# Every GPU step has its own time limit; the first failure ends the script.
#   gpurun --timeout 900 -- 'bash tools/gpu_round.sh'
# STAGE=tests|bench|all; TESTS="tests/..." narrows the suite.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp PYTHONUNBUFFERED=1
OUT=gpurun_out/round
mkdir -p $OUT
STAGE=${STAGE:-all}
if [ "$STAGE" = all ] || [ "$STAGE" = tests ]; then
  timeout -k 10 600 python -u -m pytest ${TESTS:-tests} -m gpu -x -v -p no:cacheprovider --timeout 200 --timeout-method thread \
    > $OUT/pytest_gpu.log 2>&1 || { echo "TESTS_FAIL rc=$?"; grep -E "FAIL|Error|assert" $OUT/pytest_gpu.log | tail -30; exit 1; }
  tail -1 $OUT/pytest_gpu.log
fi
if [ "$STAGE" = all ] || [ "$STAGE" = bench ]; then
  timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo "SMOKE_FAIL rc=$?"; tail -5 $OUT/smoke.log; exit 1; }
  tail -1 $OUT/smoke.log
  timeout -k 10 300 python bench.py > $OUT/bench.log 2>&1 || { echo "BENCH_FAIL rc=$?"; tail -20 $OUT/bench.log; exit 1; }
  tail -1 $OUT/bench.log
fi
echo round-done
