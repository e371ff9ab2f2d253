# Summaries of tools/gpu_r06_profile.sh's passes into profiles/r06/ (here, after
# the gpurun call merged gpurun_out/prof_*): the headline and the digest-matched
# figures bench.py reads (profiles/traffic*.json).
set -e
cd "$(dirname "$0")/.."
T=${TAG:-r06}
python3 tools/summarize_profile.py $T --prof-dir gpurun_out/prof_c3 > /dev/null
python3 tools/summarize_profile.py $T --prof-dir gpurun_out/prof_stress \
  --kernel 'void wfpt::engine_kernel<3, false, 0>' --trials 250000 --name pmc_stress_engine \
  --traffic-out traffic_stress.json > /dev/null
python3 tools/summarize_profile.py $T --prof-dir gpurun_out/prof_c2 \
  --kernel 'void wfpt::direct_kernel<false, 0>' --trials 10000000 --name pmc_c2 \
  --traffic-out traffic_c2.json > /dev/null
# node level 0 of an 8-table call: 800k trials; algorithmic bytes per trial:
# x (8) + node id (4) + the term out (8)
python3 tools/summarize_profile.py $T --prof-dir gpurun_out/prof_nodes8 \
  --kernel 'void wfpt::node_fast_kernel<3, false>' --trials 800000 --bytes-per-trial 20 \
  --name pmc_node_fast8 --no-traffic > /dev/null
for f in pmc_summary pmc_stress_engine pmc_c2 pmc_node_fast8; do
  python3 -c "
import json; d = json.load(open('profiles/$T/$f.json'))
print('$f', d['kernel'], 'us %.1f' % (d['kernel_avg_ns'] / 1e3), 'fp64/trial %.0f' % d['fp64_lane_ops_per_trial'],
      'valu/trial %.0f' % d['valu_lane_ops_per_trial'], 'issue %.3f' % (d['valu_issue_utilisation'] or 0),
      'traffic x%.2f' % (d['hbm_bytes_per_launch'] / d['algorithmic_bytes_per_launch']),
      'frac %.3f' % (d['fp64_lane_ops_per_s'] / 39.3e12), 'sha', d['src_sha1'][:8])"
done
