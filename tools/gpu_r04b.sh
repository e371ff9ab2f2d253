# GPU suite, then the stress A/B (tools/gpu_stress_ab.sh), then a short bench.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r04
export PYTHONUNBUFFERED=1
timeout -k 10 1000 python -u -m pytest tests -m gpu -v -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/r04/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -3 gpurun_out/r04/pytest_gpu.log; grep -E "^FAILED" gpurun_out/r04/pytest_gpu.log | head
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
mkdir -p gpurun_out/r04/ab
timeout -k 10 900 python -u tools/ab_variants.py run --reps 3 --names default,estrin,oclmlog,zshfl > gpurun_out/r04/ab/variants.log 2>&1 || { echo AB_FAIL; tail -5 gpurun_out/r04/ab/variants.log; exit 1; }
grep SUMMARY gpurun_out/r04/ab/variants.log
for rep in 1 2; do
  for v in default cdfg1 cdfg2 cdfg8; do
    L=hddm_amd/lib/variants/lib_$v.so; [ $v = default ] && L=hddm_amd/lib/libwfpt_amd.so
    WFPT_AMD_LIB=$L timeout -k 10 120 python -u tools/cdf_probe.py --reps 10 > gpurun_out/r04/ab/cdf_$v.$rep.log 2>&1 || { echo "CDF_FAIL $v"; exit 1; }
    echo "cdf $v $rep $(cut -c1-160 gpurun_out/r04/ab/cdf_$v.$rep.log | tr '\n' ' ')"
  done
done
timeout -k 10 400 python -u bench.py --steps 20 --warmup 3 --cpu-seconds 5 > gpurun_out/r04/bench.log 2>&1 || { echo "BENCH_FAIL rc=$?"; exit 1; }
tail -1 gpurun_out/r04/bench.log | cut -c1-300
