# PMC counters (SQ/VALU) + kernel trace for several library variants on the bench.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
for v in ${VARIANTS:-default}; do
  OUT=gpurun_out/pmc_$v; mkdir -p $OUT
  export WFPT_AMD_LIB=$PWD/hddm_amd/lib/variants/libwfpt_$v.so
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o trace -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-stress > $OUT/trace.log 2>&1 || { echo "TRACE_FAIL $v rc=$?"; exit 1; }
  timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_SALU SQ_WAIT_INST_ANY SQ_WAIT_ANY --output-format csv -d $OUT/sq -o sq -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-stress > $OUT/sq.log 2>&1 || { echo "SQ_FAIL $v rc=$?"; exit 1; }
  timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_TRANS_F64 GRBM_GUI_ACTIVE --output-format csv -d $OUT/f64 -o f64 -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-stress > $OUT/f64.log 2>&1 || { echo "F64_FAIL $v rc=$?"; exit 1; }
  echo "done $v"
done
