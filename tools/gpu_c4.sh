# Config 4 at size: hierarchical HDDM 200 x 500, sample(2000) after burn-in,
# simple and full DDM (run via gpurun).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/c4
mkdir -p $O
timeout -k 10 300 python -u tools/bench_hier.py --iters 2000 --burn 500 --progress 250 --json $O/hier_simple.json > $O/simple.log 2>&1 || { echo "SIMPLE_FAIL rc=$?"; tail -5 $O/simple.log; exit 1; }
tail -1 $O/simple.log | cut -c1-600
timeout -k 10 600 python -u tools/bench_hier.py --full --iters 2000 --burn 1000 --progress 250 --json $O/hier_full.json > $O/full.log 2>&1 || { echo "FULL_FAIL rc=$?"; tail -5 $O/full.log; exit 1; }
tail -1 $O/full.log | cut -c1-900
