# Interleaved A/B of the library variants built by tools/ab_variants.py build
# (run via gpurun): REPS reps, every variant in its own process per rep.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp PYTHONUNBUFFERED=1
O=gpurun_out/ab
mkdir -p $O
timeout -k 10 ${AB_TIMEOUT:-600} python -u tools/ab_variants.py run --reps ${REPS:-3} ${NAMES:+--names $NAMES} > $O/ab.log 2>&1 || { echo "AB_FAIL rc=$?"; tail -20 $O/ab.log; exit 1; }
cut -c1-400 $O/ab.log
echo ab-done
