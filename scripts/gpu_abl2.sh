# fused-kernel ablations (diagnostic library): assign+stats and predict time per KM_ABLATE value (c3_small)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for V in ${VALS:-0 1 2 3 4}; do
  KM_ABLATE=$V timeout -k 10 120 python -u scripts/small_probe.py ${CFG:-c3_small} ${NROWS:-} --diag 2>&1 | tail -1 | sed "s/^/ABL=$V /" || exit 1
done
