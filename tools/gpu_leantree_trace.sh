set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/lt
WFPT_LEAN_TREE=1.0 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/lt/trace1 -o t -- python3 tools/stress_probe.py --reps 3 > gpurun_out/lt/t1.log 2>&1 || { echo T1_FAIL; exit 1; }
WFPT_LEAN_TREE=0 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/lt/trace0 -o t -- python3 tools/stress_probe.py --reps 3 > gpurun_out/lt/t0.log 2>&1 || { echo T0_FAIL; exit 1; }
echo done
