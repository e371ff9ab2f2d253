# The r05 profile summaries from the two round-end GPU calls (tools/gpu_final.sh,
# tools/gpu_final2.sh + the C2 pass): run here after both calls returned.
set -e
T=${TAG:-r05}
python tools/summarize_profile.py $T
python tools/summarize_profile.py $T --prof-dir gpurun_out/prof_stress --name pmc_stress_engine --kernel 'void wfpt::engine_kernel<3, false, 0>' --trials 250000 --traffic-out traffic_stress.json
python tools/summarize_profile.py $T --prof-dir gpurun_out/prof_nodes --name pmc_node_fast --kernel 'void wfpt::node_fast_kernel<3, false>' --trials 100000 --bytes-per-trial 16 --no-traffic
python tools/summarize_profile.py $T --prof-dir gpurun_out/prof_nodes --name pmc_node_chunk --kernel 'void wfpt::node_chunk_kernel<3, false>' --trials 100000 --bytes-per-trial 16 --no-traffic
python tools/summarize_profile.py $T --prof-dir gpurun_out/prof_nodes --name pmc_segment_publish --kernel 'wfpt::segment_publish_kernel' --trials 100000 --bytes-per-trial 8 --no-traffic
python tools/summarize_profile.py $T --prof-dir gpurun_out/prof_cdf --name pmc_cdf --kernel 'void wfpt::(anonymous namespace)::dmat_cdf_kernel<4>' --trials 100000 --bytes-per-trial 16 --no-traffic
python tools/summarize_profile.py $T --prof-dir gpurun_out/prof_cdf --name pmc_cdf_wave --kernel 'wfpt::(anonymous namespace)::cdf_wave_kernel' --trials 100000 --bytes-per-trial 16 --no-traffic
python tools/summarize_profile.py $T --prof-dir gpurun_out/prof_c2 --name pmc_c2 --kernel 'void wfpt::direct_kernel<false, 0>' --trials 10000000 --bytes-per-trial 8 --no-traffic
mkdir -p profiles/$T/final
cp gpurun_out/final/pytest_gpu.log gpurun_out/final/smoke.log profiles/$T/final/
tail -1 gpurun_out/final/bench.log > profiles/$T/final/bench_line.json
cp gpurun_out/final/hier_simple.json gpurun_out/final/hier_full.json gpurun_out/final/rows.jsonl gpurun_out/final/stress.log profiles/$T/final/
cp gpurun_out/prof_nodes/plain.log profiles/$T/final/node_call_probe.log
cp gpurun_out/prof_cdf/plain.log profiles/$T/final/cdf_probe.log
cp gpurun_out/prof_c2/plain.log profiles/$T/final/c2_probe.log
for f in pmc_summary pmc_c2 pmc_stress_engine pmc_node_fast pmc_node_chunk pmc_segment_publish pmc_cdf pmc_cdf_wave; do
  python3 -c "
import json; d=json.load(open('profiles/$T/$f.json')); print('$f', d['src_sha1'][:7], round(d['kernel_avg_ns']/1e3,2),'us', 'fp64/trial', round(d['fp64_lane_ops_per_trial'],1), 'valu/trial', round(d['valu_lane_ops_per_trial'],1), 'issue', round(d['valu_issue_utilisation'],3), 'frac', round(d['fp64_lane_ops_per_s']/39.3e12,3), 'hbm/alg', round(d['hbm_bytes_per_launch']/d['algorithmic_bytes_per_launch'],2))"
done
