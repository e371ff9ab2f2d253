# Round-end evidence in one call (run via gpurun): GPU suite, smoke, bench,
# rocprofv3 passes over the headline bench (tools/gpu_final2.sh: the rest).
# Each GPU step has its own limit; the first failure ends the script.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/final
mkdir -p $O
timeout -k 10 700 python -u -m pytest tests -m gpu -v -p no:cacheprovider --timeout 200 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo "TESTS_FAIL rc=$?"; grep -E "FAIL|Error" $O/pytest_gpu.log | tail -20; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "SMOKE_FAIL rc=$?"; tail -5 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 300 python bench.py > $O/bench.log 2>&1 || { echo "BENCH_FAIL rc=$?"; tail -5 $O/bench.log; exit 1; }
tail -1 $O/bench.log | cut -c1-240
bash tools/gpu_profile.sh || exit 1
echo final-done
