# Node path grids: node tests, seed-3 slow call, node latency, config 4 full + simple.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1
O=gpurun_out/r04k
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_parity_trials.py tests/test_gpu_parity.py tests/test_parity_summing.py -m gpu -v -p no:cacheprovider --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo "PYTEST_FAIL rc=$?"; tail -5 $O/pytest_gpu.log; grep -E "^FAILED" $O/pytest_gpu.log | head; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 180 python -u tools/slow_node_probe.py tools/scratch/slow_seed3.npz > $O/slow_probe.log 2>&1 || { echo PROBE_FAIL; exit 1; }
cut -c1-120 $O/slow_probe.log
timeout -k 10 300 python -u tools/bench_node_latency.py --reps 2000 --json $O/node_latency.json > $O/node_latency.log 2>&1 || { echo NODE_FAIL; exit 1; }
timeout -k 10 300 python -u tools/bench_hier.py --full --iters 2000 --burn 1000 --dt 1e-4 --progress 500 --watchdog 280 --json $O/hier_full.json > $O/hier_full.log 2>&1 || { echo HIER_FAIL; exit 1; }
timeout -k 10 300 python -u tools/bench_hier.py --iters 2000 --burn 500 --dt 1e-4 --progress 500 --watchdog 280 --json $O/hier_simple.json > $O/hier_simple.log 2>&1 || { echo HIER_FAIL; exit 1; }
python -c "
import json
for f in ('hier_full','hier_simple'):
    d=json.load(open('$O/'+f+'.json')); print(f, d['seconds'], d['device_per_call']['v'])"
echo r04k-done
