# Stall-attribution PMC passes (wait / issue-stall / active / ifetch / smem /
# lane activity) of the headline bench for each library variant in $VARIANTS
# (hddm_amd/lib/variants/libwfpt_<name>.so; "main" = the default library).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
for v in ${VARIANTS:-main}; do
  OUT=gpurun_out/stall${TAG:-}/$v
  rm -rf $OUT; mkdir -p $OUT
  if [ "$v" = main ]; then unset WFPT_AMD_LIB; else export WFPT_AMD_LIB=$PWD/hddm_amd/lib/variants/libwfpt_$v.so; fi
  B="${CMD:-python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-stress}"
  timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o trace -- $B > $OUT/trace.log 2>&1 || { echo "TRACE_FAIL $v"; exit 1; }
  timeout -k 10 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_IFETCH SQ_INSTS_SMEM SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_VALU --output-format csv -d $OUT/p1 -o p1 -- $B > $OUT/p1.log 2>&1 || { echo "P1_FAIL $v"; exit 1; }
  timeout -k 10 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_BRANCH SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_SMEM SQ_INSTS_VSKIPPED SQ_WAVES SQ_BUSY_CYCLES --output-format csv -d $OUT/p2 -o p2 -- $B > $OUT/p2.log 2>&1 || { echo "P2_FAIL $v"; exit 1; }
  echo "stall $v done"
done
