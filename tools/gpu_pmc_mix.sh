# Instruction-mix PMC passes for the headline kernel (one rocprofv3 pass each).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/mix
mkdir -p $O
B="python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline"
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_VALU_CVT SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_TRANS_F32 --output-format csv -d $O/a -o a -- $B > $O/a.log 2>&1 || { echo "A_FAIL"; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_INSTS_SALU SQ_WAIT_ANY --output-format csv -d $O/b -o b -- $B > $O/b.log 2>&1 || { echo "B_FAIL"; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_BRANCH SQ_INSTS_SMEM SQ_INSTS_VMEM SQ_INSTS_VSKIPPED GRBM_GUI_ACTIVE --output-format csv -d $O/c -o c -- $B > $O/c.log 2>&1 || { echo "C_FAIL"; exit 1; }
echo done
