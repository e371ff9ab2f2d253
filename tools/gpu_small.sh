set -o pipefail
cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 180 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_gpu.log; grep -E "FAILED|Error" gpurun_out/pytest_gpu.log | head -5
[ $rc -eq 0 ] || exit 1
WFPT_SMALL=0 timeout -k 10 300 python -u tools/bench_node_latency.py --reps 2000 --json gpurun_out/lat_nosmall.json > gpurun_out/lat_nosmall.log 2>&1 || exit 1
timeout -k 10 300 python -u tools/bench_node_latency.py --reps 2000 --json gpurun_out/lat_small.json > gpurun_out/lat_small.log 2>&1 || exit 1
python3 - <<'PY'
import json
for f in ("lat_nosmall","lat_small"):
    d=json.load(open(f"gpurun_out/{f}.json"))
    print(f, {fam:{k:round(v["median_us"],1) for k,v in r.items() if isinstance(v,dict) and "median_us" in v} for fam,r in d["rows"].items()})
PY
