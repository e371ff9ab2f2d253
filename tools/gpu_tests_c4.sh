# GPU suite, then the config-4 per-update call costs (run via gpurun).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/tc
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/tc/pytest.log 2>&1 || { echo "TESTS_FAIL rc=$?"; grep -E "FAIL|Error|assert" gpurun_out/tc/pytest.log | tail -30; exit 1; }
tail -2 gpurun_out/tc/pytest.log
bash tools/gpu_c4_calls.sh
