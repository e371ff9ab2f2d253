set -o pipefail
cd "$GRAFT_REPO_ROOT"
for v in ${VARIANTS:-default}; do
  echo "== $v"
  WFPT_AMD_LIB=$PWD/hddm_amd/lib/variants/libwfpt_$v.so timeout -k 10 200 python -u tools/size_probe.py --reps 10 || exit 1
done
