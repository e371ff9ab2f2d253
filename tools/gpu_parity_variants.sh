# GPU: parity tests against each build variant (WFPT_AMD_LIB), then A/B timing.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for v in ${VARIANTS:-default guard}; do
  WFPT_AMD_LIB=$PWD/hddm_amd/lib/variants/libwfpt_$v.so timeout -k 10 600 python -m pytest tests -m gpu -q -p no:cacheprovider --timeout 240 -x > gpurun_out/pytest_$v.log 2>&1; rc=$?
  echo "pytest[$v] rc=$rc $(tail -1 gpurun_out/pytest_$v.log)"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
done
timeout -k 10 900 python tools/ab_variants.py run --reps ${REPS:-3} > gpurun_out/ab.log 2>&1 || { echo "AB_FAIL rc=$?"; tail -5 gpurun_out/ab.log; exit 1; }
grep SUMMARY gpurun_out/ab.log
