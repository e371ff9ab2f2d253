# r04 final build, part A: GPU suite, headline roofline passes
# (tools/gpu_profile.sh -> profiles/traffic.json), C2 and CDF PMC passes.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1
O=gpurun_out/final
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -v -p no:cacheprovider --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo "PYTEST_FAIL rc=$?"; tail -5 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
bash tools/gpu_profile.sh || { echo PROFILE_FAIL; exit 1; }
OUT=prof_c2 CMD="python3 tools/c2_probe.py --reps 20" bash tools/gpu_profile_cmd.sh || { echo C2_PROF_FAIL; exit 1; }
OUT=prof_cdf CMD="python3 tools/cdf_probe.py --reps 10" bash tools/gpu_profile_cmd.sh || { echo CDF_PROF_FAIL; exit 1; }
echo final-a-done
