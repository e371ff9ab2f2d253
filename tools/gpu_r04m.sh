# Full-DDM split small kernel: node-sized parity tests, per-node latency A/B.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1
O=gpurun_out/r04m
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_parity_summing.py tests/test_parity_strict.py tests/test_parity_trials.py -m gpu -v -p no:cacheprovider --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo "PYTEST_FAIL rc=$?"; tail -5 $O/pytest_gpu.log; grep -E "^FAILED" $O/pytest_gpu.log | head; exit 1; }
tail -1 $O/pytest_gpu.log
for rep in 1 2; do
  for v in default split2 nosplit; do
    L=hddm_amd/lib/variants/lib_$v.so; [ $v = default ] && L=hddm_amd/lib/libwfpt_amd.so
    WFPT_AMD_LIB=$L timeout -k 10 200 python -u tools/bench_node_latency.py --reps 1000 --json $O/lat_$v.$rep.json > $O/lat_$v.$rep.log 2>&1 || { echo "LAT_FAIL $v"; tail -3 $O/lat_$v.$rep.log; exit 1; }
    python -c "
import json; d=json.load(open('$O/lat_$v.$rep.json'))
print('$v', $rep, {f: (r['capi_resident']['median_us'], r['wfpt_like_res']['median_us']) for f, r in d['rows'].items()})"
  done
done
echo r04m-done
