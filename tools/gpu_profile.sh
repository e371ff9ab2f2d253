# rocprofv3 passes for the headline bench (run via gpurun). Trace+stats first,
# then one PMC group per pass (never combined with tracing domains).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/prof
mkdir -p $OUT
rm -rf $OUT/trace $OUT/fetch $OUT/write $OUT/sq $OUT/f64
# the source digest of the library these passes measure (summarize_profile.py
# ties the summary to it)
cp hddm_amd/lib/libwfpt_amd.so.src $OUT/src_sha1.txt
B="python3 bench.py --steps ${STEPS:-20} --warmup 2 --no-cpu-baseline --no-stress ${BENCH_ARGS:-}"
timeout -k 10 300 python3 bench.py --steps 30 --warmup 3 --cpu-seconds 10 > $OUT/bench_plain.log 2>&1 || { echo "BENCH_FAIL rc=$?"; exit 1; }
echo bench-ok
rocprofv3 -L > $OUT/counters_list.txt 2>&1 || true
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o trace -- $B > $OUT/trace_bench.log 2>&1 || { echo "TRACE_FAIL rc=$?"; exit 1; }
echo trace-ok
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch -o fetch -- $B > $OUT/fetch.log 2>&1 || { echo "FETCH_FAIL rc=$?"; exit 1; }
echo fetch-ok
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/write -o write -- $B > $OUT/write.log 2>&1 || { echo "WRITE_FAIL rc=$?"; exit 1; }
echo write-ok
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_SALU GRBM_GUI_ACTIVE --output-format csv -d $OUT/sq -o sq -- $B > $OUT/sq.log 2>&1 || { echo "SQ_FAIL rc=$?"; exit 1; }
echo sq-ok
F64=$(grep -oE "SQ_INSTS_VALU_[A-Z_]*F64" $OUT/counters_list.txt | sort -u | head -6 | tr '\n' ' ')
echo "f64 counters: $F64"
if [ -n "$F64" ]; then
  timeout -k 10 300 rocprofv3 --pmc $F64 --output-format csv -d $OUT/f64 -o f64 -- $B > $OUT/f64.log 2>&1 || echo "F64_FAIL rc=$?"
fi
echo done
