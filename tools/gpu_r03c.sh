# parity suite on the current build, A/B of the variants, config-4 slow-call capture + replay
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/hier
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 180 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 600 python -u tools/ab_variants.py run --reps 3 > gpurun_out/ab.log 2>&1 || { echo "AB_FAIL"; tail -5 gpurun_out/ab.log; exit 1; }
grep SUMMARY gpurun_out/ab.log
timeout -k 10 170 python -u tools/bench_hier.py --full --iters 10 --burn 50 --dt 1e-4 --seed 3 --progress 10 --watchdog 150 --slow-dump gpurun_out/hier/slow_seed3.npz > gpurun_out/hier/slow_seed3.log 2>&1; echo "slow-dump rc=$?"
timeout -k 10 120 python -u tools/slow_node_probe.py gpurun_out/hier/slow_seed3.npz --reps 3 > gpurun_out/hier/slow_probe.log 2>&1 || { echo PROBE_FAIL; tail -20 gpurun_out/hier/slow_probe.log; exit 1; }
tail -1 gpurun_out/hier/slow_probe.log
