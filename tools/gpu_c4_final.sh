set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/final3
mkdir -p $O
timeout -k 10 300 python -u tools/bench_hier.py --full --iters 2000 --burn 1000 --dt 1e-4 --progress 500 --watchdog 280 --json $O/hier_full.json > $O/hier_full.log 2>&1 || { echo HIER_FAIL; exit 1; }
timeout -k 10 300 python -u tools/bench_hier.py --iters 2000 --burn 500 --dt 1e-4 --progress 500 --watchdog 280 --json $O/hier_simple.json > $O/hier_simple.log 2>&1 || { echo HIER_FAIL; exit 1; }
timeout -k 10 300 python -u tools/bench_hier.py --full --iters 2000 --burn 1000 --dt 1e-4 --p-outlier 0 --progress 500 --watchdog 280 --json $O/hier_full_po0.json > $O/hier_full_po0.log 2>&1 || { echo HIER_FAIL; exit 1; }
echo c4-done
