# Headline + config-4 + rows on the current build (run via gpurun).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/numbers
mkdir -p $O
timeout -k 10 300 python bench.py > $O/bench.log 2>&1 || { echo "BENCH_FAIL rc=$?"; tail -5 $O/bench.log; exit 1; }
tail -1 $O/bench.log | cut -c1-200
timeout -k 10 300 python -u tools/bench_hier.py --iters 2000 --burn 500 --progress 500 --json $O/hier_simple.json > $O/hier_simple.log 2>&1 || { echo "HSIMPLE_FAIL rc=$?"; exit 1; }
timeout -k 10 600 python -u tools/bench_hier.py --full --iters 2000 --burn 1000 --progress 500 --json $O/hier_full.json > $O/hier_full.log 2>&1 || { echo "HFULL_FAIL rc=$?"; exit 1; }
timeout -k 10 500 python -u tools/bench_rows.py > $O/rows.jsonl 2> $O/rows.err || { echo "ROWS_FAIL rc=$?"; exit 1; }
timeout -k 10 300 python tools/stress_probe.py > $O/stress.log 2>&1 || { echo "STRESS_FAIL rc=$?"; exit 1; }
timeout -k 10 200 python tools/allreduce_probe.py > $O/allreduce.log 2>&1 || { echo "AR_FAIL rc=$?"; exit 1; }
tail -1 $O/stress.log; tail -1 $O/allreduce.log
