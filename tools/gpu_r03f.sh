set -o pipefail
cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python -u tools/ab_variants.py run --reps 3 --names ${NAMES:-default,l0u,prev} > gpurun_out/ab.log 2>&1 || { echo "AB_FAIL"; tail -5 gpurun_out/ab.log; exit 1; }
grep SUMMARY gpurun_out/ab.log
for v in ${NAMES_NODES:-default l0u prev}; do
  WFPT_AMD_LIB=$PWD/hddm_amd/lib/variants/libwfpt_$v.so timeout -k 10 200 python -u tools/bench_nodes.py > gpurun_out/nodes_$v.log 2>&1 || { echo NODES_FAIL; exit 1; }
  echo "nodes $v:"; cat gpurun_out/nodes_$v.log
done
