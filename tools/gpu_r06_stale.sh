# Evidence for the node publication's ordering (VERDICT r05 "do this" 1): the
# staleness check on the shipped library and on the WFPT_PUB_DIAG build
# (sums stored after the completion word), each once; JSON lines under
# gpurun_out/stale_diag/ (copied to profiles/r06/stale_diag/).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/stale_diag
mkdir -p $O
for full in "" "--full"; do
  timeout -k 10 180 python -u tests/node_publication_check.py $full --reps 400 >> $O/shipped.jsonl 2> $O/shipped.err || { echo "SHIPPED_FAIL rc=$?"; tail -5 $O/shipped.err; exit 1; }
done
WFPT_AMD_LIB=hddm_amd/lib/libwfpt_amd_pubdiag.so timeout -k 10 180 python -u tests/node_publication_check.py --full --reps 40 > $O/pubdiag.jsonl 2> $O/pubdiag.err || { echo "DIAG_FAIL rc=$?"; tail -5 $O/pubdiag.err; exit 1; }
cat $O/shipped.jsonl $O/pubdiag.jsonl
