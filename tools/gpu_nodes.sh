# Node-path iteration (one gpurun call): node / hierarchical GPU tests, the
# batched node call with and without the t-node split (and its kernel
# trace), then optionally (HIER=1) config 4's sample(2000) full and simple.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp PYTHONUNBUFFERED=1
O=gpurun_out/nodes
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_parity_trials.py tests/test_hierarchical.py tests/test_parity_summing.py tests/test_dist.py -m gpu -x -v -p no:cacheprovider --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { echo "TESTS_FAIL rc=$?"; grep -E "FAIL|Error|assert" $O/pytest.log | tail -30; exit 1; }
tail -1 $O/pytest.log
for sp in 0 1; do
  WFPT_NODE_SPLIT=$sp timeout -k 10 200 python -u tools/node_call_probe.py --reps 300 > $O/probe_${sp}.log 2>&1 || { echo "PROBE_FAIL rc=$?"; tail -5 $O/probe_${sp}.log; exit 1; }
  cut -c1-220 $O/probe_${sp}.log
  rm -rf $O/trace_$sp
  WFPT_NODE_SPLIT=$sp timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_$sp -o t -- python3 tools/node_call_probe.py --reps 100 > $O/trace_$sp.log 2>&1 || { echo "TRACE_FAIL rc=$?"; exit 1; }
  python3 -c "
import csv,glob
f=glob.glob('$O/trace_$sp/**/*kernel_stats.csv',recursive=True)[0]
for r in list(csv.DictReader(open(f)))[:12]: print('  ', r['Name'][:70], r['Calls'], round(float(r['AverageNs'])/1e3,2), 'us')
"
done
if [ "${HIER:-0}" = 1 ]; then
  timeout -k 10 300 python -u tools/bench_hier.py --full --iters 2000 --burn 1000 --dt 1e-4 --progress 500 --watchdog 280 --json $O/hier_full.json > $O/hier_full.log 2>&1 || { echo "HIER_FAIL rc=$?"; tail -5 $O/hier_full.log; exit 1; }
  python -c "import json;d=json.load(open('$O/hier_full.json'));print('full', d['seconds'], d.get('device_per_call'))"
  timeout -k 10 300 python -u tools/bench_hier.py --iters 2000 --burn 500 --dt 1e-4 --progress 500 --watchdog 280 --json $O/hier_simple.json > $O/hier_simple.log 2>&1 || { echo "HIER_FAIL rc=$?"; tail -5 $O/hier_simple.log; exit 1; }
  python -c "import json;d=json.load(open('$O/hier_simple.json'));print('simple', d['seconds'], d.get('device_per_call'))"
fi
echo nodes-done
