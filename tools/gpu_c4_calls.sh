# Config 4 full DDM: per-update likelihood call cost (run via gpurun).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/c4c
mkdir -p $O
timeout -k 10 400 python -u tools/bench_hier.py --full --iters 300 --burn 700 --progress 250 --json $O/hier_full_calls.json > $O/full.log 2>&1 || { echo "FULL_FAIL rc=$?"; tail -5 $O/full.log; exit 1; }
python - $O/hier_full_calls.json <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
print(json.dumps(d["likelihood_calls_by_update"]))
print(json.dumps(d["device_per_call"]))
print(d["state"], d["value"], d["likelihood_fraction_of_time"])
PY
