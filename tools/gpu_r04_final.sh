# r04 final numbers on the current build: roofline passes (tools/gpu_profile.sh),
# stress, seed-3 slow-call replay, per-node latency, rows, config 4 (default
# seed, full and simple; the seed-3 chain that trapped r03's run, to its end).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1
O=gpurun_out/final
mkdir -p $O/hier
bash tools/gpu_profile.sh || { echo PROFILE_FAIL; exit 1; }
timeout -k 10 200 python -u tools/stress_probe.py --reps 10 > $O/stress.log 2>&1 || { echo STRESS_FAIL; exit 1; }
tail -1 $O/stress.log
timeout -k 10 180 python -u tools/slow_node_probe.py tools/scratch/slow_seed3.npz > $O/slow_probe.log 2>&1 || { echo PROBE_FAIL; exit 1; }
timeout -k 10 300 python -u tools/bench_node_latency.py --reps 2000 --json $O/node_latency.json > $O/node_latency.log 2>&1 || { echo NODE_FAIL; exit 1; }
echo node-latency-ok
timeout -k 10 600 python -u tools/bench_rows.py --cpu-seconds 2 > $O/rows.jsonl 2> $O/rows.err || { echo ROWS_FAIL; exit 1; }
echo rows-ok
timeout -k 10 300 python -u tools/bench_hier.py --full --iters 2000 --burn 1000 --dt 1e-4 --progress 500 --watchdog 280 --json $O/hier/hier_full.json > $O/hier/hier_full.log 2>&1 || { echo HIER_FAIL; exit 1; }
timeout -k 10 300 python -u tools/bench_hier.py --iters 2000 --burn 500 --dt 1e-4 --progress 500 --watchdog 280 --json $O/hier/hier_simple.json > $O/hier/hier_simple.log 2>&1 || { echo HIER_FAIL; exit 1; }
timeout -k 10 300 python -u tools/bench_hier.py --full --seed 3 --iters 1000 --burn 50 --dt 1e-4 --progress 100 --watchdog 280 --json $O/hier/hier_seed3.json > $O/hier/hier_seed3.log 2>&1 || { echo HIER3_FAIL; exit 1; }
echo batch-done
OUT=prof_cdf CMD="python3 tools/cdf_probe.py --reps 10 --trials 50000" bash tools/gpu_profile_cmd.sh || { echo CDF_PROF_FAIL; exit 1; }
bash tools/gpu_profile_stress.sh || { echo STRESS_PROF_FAIL; exit 1; }
echo final-done
