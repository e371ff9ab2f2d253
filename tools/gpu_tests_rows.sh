# GPU suite, then every row of tools/bench_rows.py (run via gpurun).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/tr
mkdir -p $O
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { echo "TESTS_FAIL rc=$?"; grep -E "PASS|FAIL|Error" $O/pytest.log | tail -30; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 500 python -u tools/bench_rows.py > $O/rows.jsonl 2> $O/rows.err || { echo "ROWS_FAIL rc=$?"; tail -20 $O/rows.err; exit 1; }
cut -c1-300 $O/rows.jsonl
