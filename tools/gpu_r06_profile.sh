# Round-6 rocprofv3 evidence (run via gpurun): kernel trace + stats, then one
# PMC group per pass (never combined with tracing), for four workloads:
#   c3      bench.py's headline (lean_kernel<3>, 1M C3 trials)
#   stress  the stress sets whose steady state runs engine_kernel<3>
#   c2      10M simple-DDM trials (direct_kernel)
#   nodes8  config 4's batched node call over 8 parameter tables (node_fast_kernel<3>)
# Output: gpurun_out/prof_<name>/{trace,fetch,write,sq,f64}; summarised here by
# tools/summarize_profile.py --prof-dir.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
run_passes() {  # name, command
  local OUT=gpurun_out/prof_$1
  shift
  rm -rf $OUT
  mkdir -p $OUT
  cp hddm_amd/lib/libwfpt_amd.so.src $OUT/src_sha1.txt
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o trace -- "$@" > $OUT/trace.log 2>&1 || { echo "TRACE_FAIL $OUT rc=$?"; return 1; }
  timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch -o fetch -- "$@" > $OUT/fetch.log 2>&1 || { echo "FETCH_FAIL $OUT"; return 1; }
  timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/write -o write -- "$@" > $OUT/write.log 2>&1 || { echo "WRITE_FAIL $OUT"; return 1; }
  timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_SALU GRBM_GUI_ACTIVE --output-format csv -d $OUT/sq -o sq -- "$@" > $OUT/sq.log 2>&1 || { echo "SQ_FAIL $OUT"; return 1; }
  timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64 --output-format csv -d $OUT/f64 -o f64 -- "$@" > $OUT/f64.log 2>&1 || { echo "F64_FAIL $OUT"; return 1; }
  echo "$OUT ok"
}
W=${WHICH:-c3 stress c2 nodes8}
for w in $W; do
  case $w in
    c3) run_passes c3 python3 bench.py --steps 20 --warmup 2 --no-cpu-baseline --no-stress --no-extra --no-c4 || exit 1 ;;
    stress) run_passes stress python3 tools/stress_probe.py --reps 5 --engine-only || exit 1 ;;
    c2) run_passes c2 python3 tools/c2_probe.py --reps 20 || exit 1 ;;
    nodes8) run_passes nodes8 python3 tools/node_multi_probe.py --reps 20 --tables 8 --full-only || exit 1 ;;
  esac
done
echo profile-done
