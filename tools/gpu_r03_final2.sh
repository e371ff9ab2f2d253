# final-build numbers: C5 shard (world-1 RCCL), rows, per-node latency, size scaling
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/final2
mkdir -p $O
timeout -k 10 300 python -u tools/allreduce_probe.py --trials 12500000 --steps 20 > $O/allreduce.log 2>&1 || { echo AR_FAIL; tail -5 $O/allreduce.log; exit 1; }
tail -1 $O/allreduce.log
timeout -k 10 300 python -u tools/size_probe.py --reps 10 > $O/size.log 2>&1 || { echo SIZE_FAIL; exit 1; }
cat $O/size.log
timeout -k 10 300 python -u tools/bench_node_latency.py --reps 2000 --json $O/node_latency.json > $O/node_latency.log 2>&1 || { echo NODE_FAIL; exit 1; }
echo node-ok
timeout -k 10 600 python -u tools/bench_rows.py --cpu-seconds 2 > $O/rows.jsonl 2> $O/rows.err || { echo ROWS_FAIL; exit 1; }
echo rows-ok
