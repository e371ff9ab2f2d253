# Round-end evidence, second call (run via gpurun after tools/gpu_final.sh):
# rocprofv3 trace + PMC passes over the stress sets, config 4's batched node
# call and the DMAT CDF; config-4 sample(2000) simple + full; every row; stress.
# Each GPU step has its own limit; the first failure ends the script.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/final
mkdir -p $O
bash tools/gpu_profile_stress.sh > $O/prof_stress.out 2>&1 || { echo "PSTRESS_FAIL"; tail -3 $O/prof_stress.out; exit 1; }
echo prof-stress-ok
OUT=prof_nodes CMD="python3 tools/node_call_probe.py --reps 100" bash tools/gpu_profile_cmd.sh > $O/prof_nodes.out 2>&1 || { echo "PNODES_FAIL"; tail -3 $O/prof_nodes.out; exit 1; }
echo prof-nodes-ok
OUT=prof_cdf CMD="python3 tools/cdf_probe.py --reps 10" bash tools/gpu_profile_cmd.sh > $O/prof_cdf.out 2>&1 || { echo "PCDF_FAIL"; tail -3 $O/prof_cdf.out; exit 1; }
echo prof-cdf-ok
timeout -k 10 300 python -u tools/bench_hier.py --iters 2000 --burn 500 --progress 500 --json $O/hier_simple.json > $O/hier_simple.log 2>&1 || { echo "HSIMPLE_FAIL rc=$?"; tail -5 $O/hier_simple.log; exit 1; }
timeout -k 10 600 python -u tools/bench_hier.py --full --iters 2000 --burn 1000 --progress 500 --json $O/hier_full.json > $O/hier_full.log 2>&1 || { echo "HFULL_FAIL rc=$?"; tail -5 $O/hier_full.log; exit 1; }
echo hier-ok
timeout -k 10 500 python -u tools/bench_rows.py > $O/rows.jsonl 2> $O/rows.err || { echo "ROWS_FAIL rc=$?"; tail -5 $O/rows.err; exit 1; }
timeout -k 10 300 python tools/stress_probe.py > $O/stress.log 2>&1 || { echo "STRESS_FAIL rc=$?"; exit 1; }
tail -1 $O/stress.log
echo final2-done
