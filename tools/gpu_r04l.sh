# Kernel trace of a short config-4 full run (per-kernel times of the node path).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
O=gpurun_out/r04l
mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o trace -- python3 tools/bench_hier.py --full --iters 300 --burn 100 --dt 1e-4 --progress 100 --watchdog 250 --json $O/hier.json > $O/trace.log 2>&1 || { echo TRACE_FAIL; tail -5 $O/trace.log; exit 1; }
echo r04l-done
