# config 4: correctly specified model (p_outlier 0) vs HDDM's 0.05 on the same
# data, then the seed that went silent in the r03 batch (watchdog + progress).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/hier
timeout -k 10 300 python -u tools/bench_hier.py --full --iters 2000 --burn 1000 --dt 1e-4 --p-outlier 0 --progress 250 --watchdog 280 --json gpurun_out/hier/hier_full_po0.json > gpurun_out/hier/hier_full_po0.log 2>&1 || { echo C4_FULL_FAIL; exit 1; }
timeout -k 10 300 python -u tools/bench_hier.py --iters 2000 --burn 500 --dt 1e-4 --p-outlier 0 --progress 250 --watchdog 280 --json gpurun_out/hier/hier_simple_po0.json > gpurun_out/hier/hier_simple_po0.log 2>&1 || { echo C4_SIMPLE_FAIL; exit 1; }
timeout -k 10 170 python -u tools/bench_hier.py --full --iters 1000 --burn 1000 --dt 1e-4 --seed 3 --progress 10 --watchdog 150 --json gpurun_out/hier/ident_seed3.json > gpurun_out/hier/ident_seed3.log 2>&1 || { echo SEED3_FAIL; tail -40 gpurun_out/hier/ident_seed3.log; exit 1; }
echo c4-done
