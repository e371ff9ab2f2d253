# rocprofv3 host-trap PC sampling of the headline bench (instruction-level
# time attribution of the lean kernel). Separate from PMC passes.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/pcs
rm -rf $OUT; mkdir -p $OUT
rocprofv3 -L > $OUT/avail.txt 2>&1 || true
grep -i -A3 "pc.sampl\|pc_sampl" $OUT/avail.txt | head -20
timeout -k 10 180 rocprofv3 --pc-sampling-beta-enabled --pc-sampling-method host_trap --pc-sampling-unit time --pc-sampling-interval ${PCS_INTERVAL:-1} --output-format csv -d $OUT -o pcs -- python3 bench.py --steps ${STEPS:-30} --warmup 2 --no-cpu-baseline --no-stress > $OUT/pcs.log 2>&1 || { echo "PCS_FAIL rc=$?"; tail -20 $OUT/pcs.log; exit 1; }
find $OUT -name "*.csv" | head
for f in $(find $OUT -name "*pc_sampling*.csv" | head -2); do head -3 $f; wc -l $f; done
echo pcs-done
