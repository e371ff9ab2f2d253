# Kernel-level rocprof of the CDF probe for library variants (via gpurun):
#   NAMES="base bey" bash tools/gpu_cdf_prof.sh
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp PYTHONUNBUFFERED=1
O=gpurun_out/cdf_prof
mkdir -p $O
for n in ${NAMES:-base bey}; do
  WFPT_AMD_LIB=$PWD/hddm_amd/lib/variants/libwfpt_cdf_$n.so timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$n -o run -- python3 tools/cdf_probe.py --reps 5 > $O/$n.log 2>&1 || { echo "PROF_FAIL $n rc=$?"; tail -20 $O/$n.log; exit 1; }
  f=$(find $O/$n -name '*kernel_stats.csv' | head -1)
  echo "== $n"; cut -d, -f1-8 "$f" | head -12
done
echo prof-done
