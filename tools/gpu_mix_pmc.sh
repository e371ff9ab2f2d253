# VALU instruction mix of the headline bench's lean kernel (one PMC pass)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/mix
rm -rf $OUT; mkdir -p $OUT
B="python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline"
timeout -k 10 120 rocprofv3 --pmc SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_CVT SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU --output-format csv -d $OUT/m1 -o m1 -- $B > $OUT/m1.log 2>&1 || { echo "MIX_FAIL"; exit 1; }
echo mix-done
