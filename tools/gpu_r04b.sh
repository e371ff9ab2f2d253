# GPU suite, then the stress A/B (tools/gpu_stress_ab.sh), then a short bench.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r04
export PYTHONUNBUFFERED=1
timeout -k 10 1000 python -u -m pytest tests -m gpu -v -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/r04/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -3 gpurun_out/r04/pytest_gpu.log; grep -E "^FAILED" gpurun_out/r04/pytest_gpu.log | head
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
bash tools/gpu_stress_ab.sh || exit 1
timeout -k 10 400 python -u bench.py --steps 20 --warmup 3 --cpu-seconds 5 > gpurun_out/r04/bench.log 2>&1 || { echo "BENCH_FAIL rc=$?"; exit 1; }
tail -1 gpurun_out/r04/bench.log | cut -c1-300
