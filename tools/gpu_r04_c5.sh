# C5 shard (12.5M resident trials) with the world-1 RCCL all-reduce, final build.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out/c5
for rep in 1 2; do
  timeout -k 10 300 python -u tools/allreduce_probe.py --steps 20 > gpurun_out/c5/probe.$rep.log 2>&1 || { echo C5_FAIL; tail -5 gpurun_out/c5/probe.$rep.log; exit 1; }
  tail -1 gpurun_out/c5/probe.$rep.log
done
