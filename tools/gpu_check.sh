# GPU check: smoke -> pytest -m gpu -> bench -> config-4 harness bench. Each GPU
# step has its own limit; any abort/timeout ends the script (no retries).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo "SMOKE_FAIL rc=$?"; exit 1; }
timeout -k 10 900 python -m pytest tests -m gpu -v -p no:cacheprovider --timeout 300 > gpurun_out/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 400 python bench.py --steps 20 --warmup 3 --cpu-seconds 5 > gpurun_out/bench.log 2>&1 || { echo "BENCH_FAIL rc=$?"; exit 1; }
tail -1 gpurun_out/bench.log
if [ -n "${HIER:-}" ]; then
  timeout -k 10 600 python tools/bench_hier.py --iters ${HIER_ITERS:-100} > gpurun_out/bench_hier.log 2>&1 || { echo "HIER_FAIL rc=$?"; exit 1; }
  tail -1 gpurun_out/bench_hier.log
fi
