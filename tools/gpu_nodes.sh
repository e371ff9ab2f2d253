# Node-path iteration (one gpurun call): node / hierarchical GPU tests, then
# the batched node call with and without the t-node split, then config 4's
# sample(2000) full and simple.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp PYTHONUNBUFFERED=1
O=gpurun_out/nodes
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_parity_trials.py tests/test_hierarchical.py tests/test_parity_summing.py tests/test_dist.py -m gpu -x -v -p no:cacheprovider --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { echo "TESTS_FAIL rc=$?"; grep -E "FAIL|Error|assert" $O/pytest.log | tail -30; exit 1; }
tail -1 $O/pytest.log
for r in 1 2; do
  for sp in 0 1; do
    WFPT_NODE_SPLIT=$sp timeout -k 10 200 python -u tools/node_call_probe.py --reps 300 > $O/probe_${sp}_$r.log 2>&1 || { echo "PROBE_FAIL rc=$?"; tail -5 $O/probe_${sp}_$r.log; exit 1; }
    cat $O/probe_${sp}_$r.log
  done
done
timeout -k 10 300 python -u tools/bench_hier.py --full --iters 2000 --burn 1000 --dt 1e-4 --progress 500 --watchdog 280 --json $O/hier_full.json > $O/hier_full.log 2>&1 || { echo "HIER_FAIL rc=$?"; tail -5 $O/hier_full.log; exit 1; }
python -c "import json;d=json.load(open('$O/hier_full.json'));print('full', d['seconds'], d.get('device_per_call'))"
timeout -k 10 300 python -u tools/bench_hier.py --iters 2000 --burn 500 --dt 1e-4 --progress 500 --watchdog 280 --json $O/hier_simple.json > $O/hier_simple.log 2>&1 || { echo "HIER_FAIL rc=$?"; tail -5 $O/hier_simple.log; exit 1; }
python -c "import json;d=json.load(open('$O/hier_simple.json'));print('simple', d['seconds'], d.get('device_per_call'))"
echo nodes-done
