# r03 measurement batch (after parity/bench): node latency, config 4 at
# dt=1e-4 (+ sv identifiability seeds), row benches, stress, and rocprofv3
# profiles of C2 / stress / CDF. Each GPU step under its own limit.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/hier
timeout -k 10 300 python -u tools/bench_node_latency.py --reps 2000 --json gpurun_out/node_latency.json > gpurun_out/node_latency.log 2>&1 || { echo NODE_FAIL; exit 1; }
timeout -k 10 300 python -u tools/stress_probe.py --reps 10 > gpurun_out/stress.log 2>&1 || { echo STRESS_FAIL; exit 1; }
OUT=prof_c2 CMD="python3 tools/c2_probe.py --reps 20" bash tools/gpu_profile_cmd.sh || exit 1
OUT=prof_stress CMD="python3 tools/stress_probe.py --reps 5" bash tools/gpu_profile_cmd.sh || exit 1
OUT=prof_cdf CMD="python3 tools/cdf_probe.py --reps 10" bash tools/gpu_profile_cmd.sh || exit 1
timeout -k 10 600 python -u tools/bench_rows.py --cpu-seconds 2 > gpurun_out/rows.jsonl 2> gpurun_out/rows.err || { echo ROWS_FAIL; exit 1; }
timeout -k 10 600 python -u tools/bench_hier.py --full --iters 2000 --burn 1000 --dt 1e-4 --json gpurun_out/hier/hier_full.json > gpurun_out/hier/hier_full.log 2>&1 || { echo HIER_FAIL; exit 1; }
timeout -k 10 600 python -u tools/bench_hier.py --iters 2000 --burn 500 --dt 1e-4 --json gpurun_out/hier/hier_simple.json > gpurun_out/hier/hier_simple.log 2>&1 || { echo HIER_FAIL; exit 1; }
for s in 1 2 3 4; do
  timeout -k 10 300 python -u tools/bench_hier.py --full --iters 1000 --burn 1000 --dt 1e-4 --seed $s --json gpurun_out/hier/ident_seed$s.json > gpurun_out/hier/ident_seed$s.log 2>&1 || { echo IDENT_FAIL; exit 1; }
done
echo batch-done
