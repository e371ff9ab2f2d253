# Interleaved A/B of the CDF variants built by tools/ab_cdf.py build (via gpurun).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp PYTHONUNBUFFERED=1
O=gpurun_out/ab_cdf
mkdir -p $O
timeout -k 10 ${AB_TIMEOUT:-600} python -u tools/ab_cdf.py run --reps ${REPS:-3} ${NAMES:+--names $NAMES} > $O/ab.log 2>&1 || { echo "AB_FAIL rc=$?"; tail -20 $O/ab.log; exit 1; }
sed -n '/SUMMARY/,$p' $O/ab.log
echo ab-done
