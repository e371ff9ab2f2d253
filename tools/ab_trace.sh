# A/B of library variants under rocprofv3 --kernel-trace (run via gpurun):
#   bash tools/ab_trace.sh "<probe command>" default v1 v2 ...
# Each variant (hddm_amd/lib/variants/libwfpt_<v>.so; "default" = the shipped
# library) runs the probe twice, interleaved; per-kernel averages printed.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
CMD="$1"; shift
O=gpurun_out/ab
mkdir -p $O
for rep in 1 2; do
  for v in "$@"; do
    if [ "$v" = default ]; then L=hddm_amd/lib/libwfpt_amd.so; else L=hddm_amd/lib/variants/libwfpt_$v.so; fi
    rm -rf $O/${v}_$rep
    WFPT_AMD_LIB=$L timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/${v}_$rep -o t -- $CMD > $O/${v}_$rep.log 2>&1 || { echo "FAIL $v"; tail -5 $O/${v}_$rep.log; exit 1; }
    echo "== $v rep $rep"
    grep '^{' $O/${v}_$rep.log | cut -c1-220
    f=$(ls $O/${v}_$rep/*kernel_stats.csv | head -1)
    python3 -c "
import csv
for r in csv.DictReader(open('$f')):
    if any(k in r['Name'] for k in ('node_', 'segment', 'lean', 'engine', 'direct', 'finalize')):
        print('   ', r['Name'][:56].ljust(56), r['Calls'].rjust(6), '%.1f' % (float(r['AverageNs']) / 1e3))
"
  done
done
