# Full-DDM split node fast pass: node parity tests, seed-3 call, config 4 full A/B.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1
O=gpurun_out/r04n
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_parity_trials.py tests/test_gpu_parity.py tests/test_parity_summing.py tests/test_dist.py -m gpu -v -p no:cacheprovider --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo "PYTEST_FAIL rc=$?"; tail -5 $O/pytest_gpu.log; grep -E "^FAILED" $O/pytest_gpu.log | head; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 180 python -u tools/slow_node_probe.py tools/scratch/slow_seed3.npz > $O/slow_probe.log 2>&1 || { echo PROBE_FAIL; exit 1; }
cut -c1-100 $O/slow_probe.log
for v in default nonodesplit; do
  L=hddm_amd/lib/variants/lib_$v.so; [ $v = default ] && L=hddm_amd/lib/libwfpt_amd.so
  WFPT_AMD_LIB=$L timeout -k 10 300 python -u tools/bench_hier.py --full --iters 2000 --burn 1000 --dt 1e-4 --progress 500 --watchdog 280 --json $O/hier_full_$v.json > $O/hier_full_$v.log 2>&1 || { echo HIER_FAIL; exit 1; }
  python -c "
import json; d=json.load(open('$O/hier_full_$v.json')); print('$v', d['seconds'], d['device_per_call']['v'])"
done
echo r04n-done
