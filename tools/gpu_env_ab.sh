# A/B of a runtime switch (environment variable) on the headline bench and the
# stress probe, interleaved rep by rep on one box (run via gpurun).
#   VAR=WFPT_LEAN A=0 B=1 REPS=3 gpurun -- 'bash tools/gpu_env_ab.sh'
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/envab
mkdir -p $O
VAR=${VAR:-WFPT_LEAN}; A=${A:-0}; B=${B:-1}; REPS=${REPS:-3}
if [ "${TESTS:-1}" = 1 ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread > $O/pytest.log 2>&1 || { echo "TESTS_FAIL rc=$?"; tail -30 $O/pytest.log; exit 1; }
  tail -2 $O/pytest.log
fi
for r in $(seq 1 $REPS); do
  for val in $A $B; do
    env $VAR=$val timeout -k 10 200 python bench.py --steps 50 --warmup 5 --no-cpu-baseline --no-stress > $O/bench_${val}_$r.log 2>&1 || { echo "BENCH_FAIL $val rc=$?"; tail -5 $O/bench_${val}_$r.log; exit 1; }
    python - $O/bench_${val}_$r.log $VAR=$val <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[2], "value %.4g" % d["value"], "ms/step %.4f" % d["ms_per_step"], "kernel_ms %.4f" % d["roofline"]["kernel_ms_avg"])
PY
    env $VAR=$val timeout -k 10 200 python tools/stress_probe.py > $O/stress_${val}_$r.log 2>&1 || { echo "STRESS_FAIL $val rc=$?"; tail -5 $O/stress_${val}_$r.log; exit 1; }
    echo "$VAR=$val $(tail -1 $O/stress_${val}_$r.log)"
  done
done
