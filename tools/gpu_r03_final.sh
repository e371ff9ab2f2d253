# r03 final numbers on the current build: rows, per-node latency, stress,
# config 4 (HDDM's p_outlier 0.05 and the correctly specified 0)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/final/hier
O=gpurun_out/final
timeout -k 10 300 python -u tools/bench_node_latency.py --reps 2000 --json $O/node_latency.json > $O/node_latency.log 2>&1 || { echo NODE_FAIL; exit 1; }
echo node-latency-ok
timeout -k 10 200 python -u tools/stress_probe.py --reps 10 > $O/stress.log 2>&1 || { echo STRESS_FAIL; exit 1; }
tail -1 $O/stress.log
timeout -k 10 600 python -u tools/bench_rows.py --cpu-seconds 2 > $O/rows.jsonl 2> $O/rows.err || { echo ROWS_FAIL; exit 1; }
echo rows-ok
timeout -k 10 300 python -u tools/bench_hier.py --full --iters 2000 --burn 1000 --dt 1e-4 --progress 500 --watchdog 280 --json $O/hier/hier_full.json > $O/hier/hier_full.log 2>&1 || { echo HIER_FAIL; exit 1; }
timeout -k 10 300 python -u tools/bench_hier.py --iters 2000 --burn 500 --dt 1e-4 --progress 500 --watchdog 280 --json $O/hier/hier_simple.json > $O/hier/hier_simple.log 2>&1 || { echo HIER_FAIL; exit 1; }
timeout -k 10 300 python -u tools/bench_hier.py --full --iters 2000 --burn 1000 --dt 1e-4 --p-outlier 0 --progress 500 --watchdog 280 --json $O/hier/hier_full_po0.json > $O/hier/hier_full_po0.log 2>&1 || { echo HIER_FAIL; exit 1; }
echo batch-done
