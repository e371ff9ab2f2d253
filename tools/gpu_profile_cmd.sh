# rocprofv3 kernel trace + PMC passes over an arbitrary probe command (run via
# gpurun): OUT=<dir under gpurun_out> CMD="python3 tools/..." bash tools/gpu_profile_cmd.sh
# Same pass layout as tools/gpu_profile.sh: trace+stats first, then one PMC
# group per pass (never combined with tracing domains).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/${OUT:?}
mkdir -p $OUT
rm -rf $OUT/trace $OUT/fetch $OUT/write $OUT/sq $OUT/f64
cp hddm_amd/lib/libwfpt_amd.so.src $OUT/src_sha1.txt
B="${CMD:?}"
timeout -k 10 300 $B > $OUT/plain.log 2>&1 || { echo "PLAIN_FAIL rc=$?"; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o trace -- $B > $OUT/trace.log 2>&1 || { echo "TRACE_FAIL rc=$?"; exit 1; }
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch -o fetch -- $B > $OUT/fetch.log 2>&1 || { echo "FETCH_FAIL rc=$?"; exit 1; }
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/write -o write -- $B > $OUT/write.log 2>&1 || { echo "WRITE_FAIL rc=$?"; exit 1; }
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_SALU SQ_INSTS_LDS GRBM_GUI_ACTIVE --output-format csv -d $OUT/sq -o sq -- $B > $OUT/sq.log 2>&1 || { echo "SQ_FAIL rc=$?"; exit 1; }
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_TRANS_F64 --output-format csv -d $OUT/f64 -o f64 -- $B > $OUT/f64.log 2>&1 || { echo "F64_FAIL rc=$?"; exit 1; }
echo "profile $OUT done"
