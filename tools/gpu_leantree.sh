set -o pipefail
cd "$GRAFT_REPO_ROOT"
for lt in 0 0.25 0.5 1.0; do
  echo "== WFPT_LEAN_TREE=$lt"
  WFPT_LEAN_TREE=$lt timeout -k 10 200 python -u tools/stress_probe.py --reps 5 || exit 1
done
