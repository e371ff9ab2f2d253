# GPU suite on the default library, then an interleaved A/B of prebuilt
# variants (NAMES=a,b) (run via gpurun).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/tab
mkdir -p $O
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { echo "TESTS_FAIL rc=$?"; grep -E "FAIL|Error|assert" $O/pytest.log | tail -30; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 600 python tools/ab_variants.py run --reps ${REPS:-3} --names ${NAMES:-default} > $O/ab.log 2>&1 || { echo "AB_FAIL rc=$?"; tail -5 $O/ab.log; exit 1; }
grep SUMMARY $O/ab.log
