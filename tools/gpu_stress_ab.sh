# Stress-set A/B: records sequence variants (records per wave) vs the chunk
# engine (WFPT_STATE=0), each in its own process; then a kernel trace of the
# default build. Output under gpurun_out/r04/ab.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp PYTHONUNBUFFERED=1
OUT=gpurun_out/r04/ab
mkdir -p $OUT
VARIANTS=${VARIANTS:-"default zshfl estrin"}
for rep in 1 2; do
  for v in $VARIANTS; do
    case $v in
      default) L=hddm_amd/lib/libwfpt_amd.so; E="";;
      records) L=hddm_amd/lib/libwfpt_amd.so; E="WFPT_STATE=1";;
      *) L=hddm_amd/lib/variants/lib_$v.so; E="";;
    esac
    env $E WFPT_AMD_LIB=$L timeout -k 10 200 python -u tools/stress_probe.py --reps 10 > $OUT/$v.$rep.log 2>&1 || { echo "FAIL $v rc=$?"; exit 1; }
    echo "$v $rep $(tail -1 $OUT/$v.$rep.log)"
  done
done
[ -n "${TRACE:-}" ] || exit 0
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o trace -- python3 tools/stress_probe.py --reps 5 > $OUT/trace.log 2>&1 || { echo "TRACE_FAIL rc=$?"; exit 1; }
echo trace-ok
