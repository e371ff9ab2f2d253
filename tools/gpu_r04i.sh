# CDF window tables check + VALU instruction-category passes (lean C3, C2).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
O=gpurun_out/r04i
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_cdfdif.py tests/test_gpu_parity.py -m gpu -v -p no:cacheprovider --timeout 200 --timeout-method thread > $O/pytest_cdf.log 2>&1 || { echo "PYTEST_FAIL rc=$?"; tail -5 $O/pytest_cdf.log; exit 1; }
tail -1 $O/pytest_cdf.log
for rep in 1 2; do
  timeout -k 10 120 python -u tools/cdf_probe.py --reps 10 > $O/cdf.$rep.log 2>&1 || { echo CDF_FAIL; exit 1; }
  cut -c1-200 $O/cdf.$rep.log
done
C="SQ_INSTS_VALU SQ_INSTS_VALU_CVT SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_TRANS_F32"
timeout -k 10 120 rocprofv3 --pmc $C --output-format csv -d $O/cat_lean -o cat -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline > $O/cat_lean.log 2>&1 || { echo CAT_FAIL; exit 1; }
timeout -k 10 120 rocprofv3 --pmc $C --output-format csv -d $O/cat_c2 -o cat -- python3 tools/c2_probe.py --reps 10 > $O/cat_c2.log 2>&1 || { echo CAT2_FAIL; exit 1; }
timeout -k 10 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_INSTS_VSKIPPED SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_WAVES --output-format csv -d $O/misc_lean -o misc -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline > $O/misc_lean.log 2>&1 || { echo MISC_FAIL; exit 1; }
echo r04i-done
