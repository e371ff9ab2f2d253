# r04 final build: parts A and B in one call (GPU suite, headline / C2 / CDF /
# stress PMC passes, stress and seed-3 slow-call probes).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
bash tools/gpu_r04_final_a.sh || exit 1
O=gpurun_out/final
export PYTHONUNBUFFERED=1
bash tools/gpu_profile_stress.sh || { echo STRESS_PROF_FAIL; exit 1; }
timeout -k 10 200 python -u tools/stress_probe.py --reps 10 > $O/stress.log 2>&1 || { echo STRESS_FAIL; exit 1; }
tail -1 $O/stress.log
timeout -k 10 180 python -u tools/slow_node_probe.py tools/scratch/slow_seed3.npz > $O/slow_probe.log 2>&1 || { echo PROBE_FAIL; exit 1; }
echo final-ab-done
