# r04 final build, one call: GPU suite + PMC passes (A), stress / seed-3
# probes (B), per-node latency and config 4 full / simple.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
bash tools/gpu_r04_final_ab.sh || exit 1
export PYTHONUNBUFFERED=1
O=gpurun_out/final
mkdir -p $O/hier
timeout -k 10 300 python -u tools/bench_node_latency.py --reps 2000 --json $O/node_latency.json > $O/node_latency.log 2>&1 || { echo NODE_FAIL; exit 1; }
timeout -k 10 300 python -u tools/bench_hier.py --full --iters 2000 --burn 1000 --dt 1e-4 --progress 500 --watchdog 280 --json $O/hier/hier_full.json > $O/hier/hier_full.log 2>&1 || { echo HIER_FAIL; exit 1; }
timeout -k 10 300 python -u tools/bench_hier.py --iters 2000 --burn 500 --dt 1e-4 --progress 500 --watchdog 280 --json $O/hier/hier_simple.json > $O/hier/hier_simple.log 2>&1 || { echo HIER_FAIL; exit 1; }
echo final-all-done
