# Iteration call: the whole GPU suite, the default bench line, and the batched
# node call with / without the t-node split (plus kernel traces).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp PYTHONUNBUFFERED=1
O=gpurun_out/iter
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 150 --timeout-method thread > $O/pytest.log 2>&1 || { echo "TESTS_FAIL rc=$?"; grep -E "FAIL|Error|assert" $O/pytest.log | tail -30; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 300 python bench.py --cpu-seconds 4 > $O/bench.log 2>&1 || { echo "BENCH_FAIL rc=$?"; tail -20 $O/bench.log; exit 1; }
python3 -c "
import json; d=json.loads(open('$O/bench.log').read().strip().splitlines()[-1])
print('bench', d['value'], d['ms_per_step'], d['roofline']['kernel_ms_avg'], 'stress', d['stress']['trials_per_s'], d['stress']['kernel_ms_avg'])"
for sp in 0 1; do
  WFPT_NODE_SPLIT=$sp timeout -k 10 200 python -u tools/node_call_probe.py --reps 300 > $O/probe_${sp}.log 2>&1 || { echo "PROBE_FAIL rc=$?"; tail -5 $O/probe_${sp}.log; exit 1; }
  cut -c1-330 $O/probe_${sp}.log
  rm -rf $O/trace_$sp
  WFPT_NODE_SPLIT=$sp timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_$sp -o t -- python3 tools/node_call_probe.py --reps 100 > $O/trace_$sp.log 2>&1 || { echo "TRACE_FAIL rc=$?"; exit 1; }
  python3 -c "
import csv,glob
f=glob.glob('$O/trace_$sp/**/*kernel_stats.csv',recursive=True)[0]
for r in list(csv.DictReader(open(f)))[:14]: print('  ', r['Name'][:60], r['Calls'], round(float(r['AverageNs'])/1e3,2), 'us')
"
done
rm -rf $O/trace_bench
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_bench -o t -- python3 bench.py --steps 20 --warmup 2 --no-cpu-baseline > $O/trace_bench.log 2>&1 || { echo "TRACE_FAIL rc=$?"; exit 1; }
python3 -c "
import csv,glob
f=glob.glob('$O/trace_bench/**/*kernel_stats.csv',recursive=True)[0]
for r in list(csv.DictReader(open(f)))[:10]: print('  ', r['Name'][:60], r['Calls'], round(float(r['AverageNs'])/1e3,2), 'us')
"
echo iter-done
