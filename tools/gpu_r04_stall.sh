# Stall attribution on the final build: lean (bench), C2, stress engine.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=_lean bash tools/gpu_stall_pmc.sh || exit 1
TAG=_c2 CMD="python3 tools/c2_probe.py --reps 10" bash tools/gpu_stall_pmc.sh || exit 1
TAG=_stress CMD="python3 tools/stress_probe.py --reps 3" bash tools/gpu_stall_pmc.sh || exit 1
echo stall-all-done
