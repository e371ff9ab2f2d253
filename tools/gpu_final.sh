# Round-end evidence in one call (run via gpurun): GPU suite, smoke, bench,
# rocprofv3 passes, config-4 sample(2000) simple + full, every row, stress.
# Each GPU step has its own limit; the first failure ends the script.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/final
mkdir -p $O
timeout -k 10 700 python -u -m pytest tests -m gpu -v --timeout 200 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo "TESTS_FAIL rc=$?"; grep -E "FAIL|Error" $O/pytest_gpu.log | tail -20; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "SMOKE_FAIL rc=$?"; tail -5 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 300 python bench.py > $O/bench.log 2>&1 || { echo "BENCH_FAIL rc=$?"; tail -5 $O/bench.log; exit 1; }
tail -1 $O/bench.log | cut -c1-240
bash tools/gpu_profile.sh || exit 1
timeout -k 10 300 python -u tools/bench_hier.py --iters 2000 --burn 500 --progress 500 --json $O/hier_simple.json > $O/hier_simple.log 2>&1 || { echo "HSIMPLE_FAIL rc=$?"; tail -5 $O/hier_simple.log; exit 1; }
timeout -k 10 600 python -u tools/bench_hier.py --full --iters 2000 --burn 1000 --progress 500 --json $O/hier_full.json > $O/hier_full.log 2>&1 || { echo "HFULL_FAIL rc=$?"; tail -5 $O/hier_full.log; exit 1; }
echo hier-ok
timeout -k 10 500 python -u tools/bench_rows.py > $O/rows.jsonl 2> $O/rows.err || { echo "ROWS_FAIL rc=$?"; tail -5 $O/rows.err; exit 1; }
timeout -k 10 300 python tools/stress_probe.py > $O/stress.log 2>&1 || { echo "STRESS_FAIL rc=$?"; exit 1; }
tail -1 $O/stress.log
