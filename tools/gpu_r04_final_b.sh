# r04 final build, part B: stress-engine PMC passes, stress / seed-3 slow-call /
# node-latency probes, the rows table.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1
O=gpurun_out/final
mkdir -p $O
bash tools/gpu_profile_stress.sh || { echo STRESS_PROF_FAIL; exit 1; }
timeout -k 10 200 python -u tools/stress_probe.py --reps 10 > $O/stress.log 2>&1 || { echo STRESS_FAIL; exit 1; }
tail -1 $O/stress.log
timeout -k 10 180 python -u tools/slow_node_probe.py tools/scratch/slow_seed3.npz > $O/slow_probe.log 2>&1 || { echo PROBE_FAIL; exit 1; }
timeout -k 10 300 python -u tools/bench_node_latency.py --reps 2000 --json $O/node_latency.json > $O/node_latency.log 2>&1 || { echo NODE_FAIL; exit 1; }
echo node-latency-ok
timeout -k 10 500 python -u tools/bench_rows.py --cpu-seconds 2 > $O/rows.jsonl 2> $O/rows.err || { echo ROWS_FAIL; exit 1; }
echo final-b-done
