# Quick GPU iteration: parity subset -> A/B of prebuilt variants (AB=names) ->
# bench -> kernel trace. Every GPU step has its own limit; failures end it.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/quick
O=gpurun_out/quick
timeout -k 10 400 python -m pytest tests -m gpu -q -x -p no:cacheprovider --timeout 200 > $O/pytest.log 2>&1 || { echo "PYTEST_FAIL rc=$?"; tail -20 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
if [ -n "${AB:-}" ]; then
  timeout -k 10 500 python tools/ab_variants.py run --reps ${REPS:-3} --names $AB > $O/ab.log 2>&1 || { echo "AB_FAIL rc=$?"; exit 1; }
  grep SUMMARY $O/ab.log
fi
timeout -k 10 300 python bench.py --steps 30 --warmup 3 --cpu-seconds 3 > $O/bench.log 2>&1 || { echo "BENCH_FAIL rc=$?"; exit 1; }
tail -1 $O/bench.log | cut -c1-400
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o trace -- python3 bench.py --steps 20 --warmup 2 --no-cpu-baseline > $O/trace.log 2>&1 || { echo "TRACE_FAIL rc=$?"; exit 1; }
head -6 $O/trace/trace_kernel_stats.csv | cut -c1-160
