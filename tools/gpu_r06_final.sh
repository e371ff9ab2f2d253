# Round-6 evidence in one call (run via gpurun): GPU suite, smoke, the default
# bench line (headline + stress + c2 + c5_n1 + c4), the node-call probes, the
# 8-chain config-4 runs and the publication staleness check. Each GPU step has
# its own limit; the first failure ends the script. Output: gpurun_out/final/.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/final
mkdir -p $O
cp hddm_amd/lib/libwfpt_amd.so.src $O/src_sha1.txt
timeout -k 10 700 python -u -m pytest tests -m gpu -v -p no:cacheprovider --timeout 240 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo "TESTS_FAIL rc=$?"; grep -E "FAIL|Error" $O/pytest_gpu.log | tail -20; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "SMOKE_FAIL rc=$?"; tail -5 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 600 python -u bench.py > $O/bench.log 2>&1 || { echo "BENCH_FAIL rc=$?"; tail -5 $O/bench.log; exit 1; }
tail -1 $O/bench.log | cut -c1-400
timeout -k 10 300 python -u tools/node_call_probe.py --reps 300 > $O/node_call_probe.log 2>&1 || { echo "PROBE_FAIL"; exit 1; }
timeout -k 10 300 python -u tools/node_multi_probe.py --reps 60 --tables 1,2,4,8,16 > $O/node_multi.log 2>&1 || { echo "MULTI_FAIL"; exit 1; }
timeout -k 10 300 python3 -u tools/bench_chains.py --chains 8 --full > $O/chains_full.json 2> $O/chains_full.err || { echo CFAIL; tail -5 $O/chains_full.err; exit 1; }
timeout -k 10 300 python3 -u tools/bench_chains.py --chains 8 > $O/chains_simple.json 2> $O/chains_simple.err || { echo SFAIL; tail -5 $O/chains_simple.err; exit 1; }
bash tools/gpu_r06_stale.sh > $O/stale.log 2>&1 || { echo STALE_FAIL; tail -5 $O/stale.log; exit 1; }
cp -r gpurun_out/stale_diag $O/
echo final-done
