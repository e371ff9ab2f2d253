# r04 final build, part C: config 4 (hierarchical sampler) runs: default seed
# full and simple, and the seed-3 chain that trapped r03's run, to its end.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1
O=gpurun_out/final/hier
mkdir -p $O
timeout -k 10 300 python -u tools/bench_hier.py --full --iters 2000 --burn 1000 --dt 1e-4 --progress 500 --watchdog 280 --json $O/hier_full.json > $O/hier_full.log 2>&1 || { echo HIER_FAIL; exit 1; }
timeout -k 10 300 python -u tools/bench_hier.py --iters 2000 --burn 500 --dt 1e-4 --progress 500 --watchdog 280 --json $O/hier_simple.json > $O/hier_simple.log 2>&1 || { echo HIER_FAIL; exit 1; }
timeout -k 10 300 python -u tools/bench_hier.py --full --seed 3 --iters 1000 --burn 50 --dt 1e-4 --progress 100 --watchdog 280 --json $O/hier_seed3.json > $O/hier_seed3.log 2>&1 || { echo HIER3_FAIL; exit 1; }
echo final-c-done
