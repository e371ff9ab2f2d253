# GPU suite, then the profile passes of tools/gpu_profile.sh (run via gpurun).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/tp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread > gpurun_out/tp/pytest.log 2>&1 || { echo "TESTS_FAIL rc=$?"; tail -30 gpurun_out/tp/pytest.log; exit 1; }
tail -2 gpurun_out/tp/pytest.log
bash tools/gpu_profile.sh
