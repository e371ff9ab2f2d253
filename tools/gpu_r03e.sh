# parity suite on the current build, A/B vs the previous build, stress probe
set -o pipefail
cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 180 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 600 python -u tools/ab_variants.py run --reps ${REPS:-3} --names ${NAMES:-default,prev} > gpurun_out/ab.log 2>&1 || { echo "AB_FAIL"; tail -5 gpurun_out/ab.log; exit 1; }
grep SUMMARY gpurun_out/ab.log
timeout -k 10 200 python -u tools/stress_probe.py --reps 5 > gpurun_out/stress.log 2>&1 || { echo STRESS_FAIL; exit 1; }
tail -1 gpurun_out/stress.log
for v in default prev; do
  WFPT_AMD_LIB=$PWD/hddm_amd/lib/variants/libwfpt_$v.so timeout -k 10 200 python -u tools/c2_probe.py --reps 20 > gpurun_out/c2_$v.log 2>&1 || { echo C2_FAIL; exit 1; }
  echo "c2 $v: $(tail -1 gpurun_out/c2_$v.log)"
done
