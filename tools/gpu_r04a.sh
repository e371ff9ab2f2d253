# r04 first GPU check: full GPU suite (new per-trial summing-path and node
# chunk-engine tests included), the seed-3 slow node call replay, a short bench.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r04
export PYTHONUNBUFFERED=1
timeout -k 10 1000 python -u -m pytest tests -m gpu -v -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/r04/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -3 gpurun_out/r04/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 180 python -u tools/slow_node_probe.py tools/scratch/slow_seed3.npz > gpurun_out/r04/slow_probe.log 2>&1 || { echo "PROBE_FAIL rc=$?"; exit 1; }
tail -2 gpurun_out/r04/slow_probe.log
timeout -k 10 400 python -u bench.py --steps 20 --warmup 3 --cpu-seconds 5 > gpurun_out/r04/bench.log 2>&1 || { echo "BENCH_FAIL rc=$?"; exit 1; }
tail -1 gpurun_out/r04/bench.log
if [ -n "${STRESS:-}" ]; then
  timeout -k 10 300 python -u tools/stress_probe.py --reps 10 --json gpurun_out/r04/stress.json > gpurun_out/r04/stress.log 2>&1 || { echo "STRESS_FAIL rc=$?"; exit 1; }
  tail -6 gpurun_out/r04/stress.log
fi
if [ -n "${STRESS_AB:-}" ]; then
  WFPT_STATE=0 timeout -k 10 300 python -u tools/stress_probe.py --reps 10 --json gpurun_out/r04/stress_nostate.json > gpurun_out/r04/stress_nostate.log 2>&1 || { echo "STRESS0_FAIL rc=$?"; exit 1; }
  tail -6 gpurun_out/r04/stress_nostate.log
fi
