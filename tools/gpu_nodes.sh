# Node-path iteration (one gpurun call): node / hierarchical GPU tests, then
# the batched node call under each variant (VARS: env assignments separated
# by spaces, e.g. "WFPT_NODE_SPEC=0 WFPT_NODE_SPEC=1") with its kernel trace,
# then optionally (HIER=1) config 4's sample(2000) full and simple.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp PYTHONUNBUFFERED=1
O=gpurun_out/nodes
mkdir -p $O
if [ "${TESTS:-1}" = 1 ]; then
timeout -k 10 400 python -u -m pytest tests/test_parity_trials.py tests/test_hierarchical.py tests/test_parity_summing.py tests/test_dist.py -m gpu -x -v -p no:cacheprovider --timeout 150 --timeout-method thread > $O/pytest.log 2>&1 || { echo "TESTS_FAIL rc=$?"; grep -E "FAIL|Error|assert" $O/pytest.log | tail -30; exit 1; }
tail -1 $O/pytest.log
fi
i=0
for v in ${VARS:-WFPT_NODE_SPLIT=0}; do
  i=$((i+1))
  env $v timeout -k 10 200 python -u tools/node_call_probe.py --reps 300 > $O/probe_$i.log 2>&1 || { echo "PROBE_FAIL rc=$?"; tail -5 $O/probe_$i.log; exit 1; }
  echo "== $v"; cut -c1-330 $O/probe_$i.log
  rm -rf $O/trace_$i
  env $v timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_$i -o t -- python3 tools/node_call_probe.py --reps 100 > $O/trace_$i.log 2>&1 || { echo "TRACE_FAIL rc=$?"; exit 1; }
  python3 tools/node_timeline.py $O/trace_$i
done
if [ "${HIER:-0}" = 1 ]; then
  timeout -k 10 300 python -u tools/bench_hier.py --full --iters 2000 --burn 1000 --dt 1e-4 --progress 500 --watchdog 280 --json $O/hier_full.json > $O/hier_full.log 2>&1 || { echo "HIER_FAIL rc=$?"; tail -5 $O/hier_full.log; exit 1; }
  python -c "import json;d=json.load(open('$O/hier_full.json'));print('full', d['seconds'], d.get('device_per_call'))"
  timeout -k 10 300 python -u tools/bench_hier.py --iters 2000 --burn 500 --dt 1e-4 --progress 500 --watchdog 280 --json $O/hier_simple.json > $O/hier_simple.log 2>&1 || { echo "HIER_FAIL rc=$?"; tail -5 $O/hier_simple.log; exit 1; }
  python -c "import json;d=json.load(open('$O/hier_simple.json'));print('simple', d['seconds'], d.get('device_per_call'))"
fi
echo nodes-done
