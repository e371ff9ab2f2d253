# Node path records/chunks hybrid: GPU suite, seed-3 slow call, config 4 full.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1
O=gpurun_out/r04j
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -v -p no:cacheprovider --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo "PYTEST_FAIL rc=$?"; tail -5 $O/pytest_gpu.log; grep -E "^FAILED" $O/pytest_gpu.log | head; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 180 python -u tools/slow_node_probe.py tools/scratch/slow_seed3.npz > $O/slow_probe.log 2>&1 || { echo PROBE_FAIL; exit 1; }
cut -c1-200 $O/slow_probe.log
timeout -k 10 300 python -u tools/bench_hier.py --full --iters 2000 --burn 1000 --dt 1e-4 --progress 500 --watchdog 280 --json $O/hier_full.json > $O/hier_full.log 2>&1 || { echo HIER_FAIL; exit 1; }
tail -1 $O/hier_full.log | cut -c1-200
echo r04j-done
