# What the driver runs at round end: smoke(), then the default bench line.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out/driver
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke-ok')" > gpurun_out/driver/smoke.log 2>&1 || { echo SMOKE_FAIL; tail -5 gpurun_out/driver/smoke.log; exit 1; }
tail -2 gpurun_out/driver/smoke.log
timeout -k 10 400 python -u bench.py > gpurun_out/driver/bench.log 2>&1 || { echo BENCH_FAIL; tail -5 gpurun_out/driver/bench.log; exit 1; }
tail -1 gpurun_out/driver/bench.log
