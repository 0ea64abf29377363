# A named subset of the GPU tests (TESTS), then an A/B of library builds
# (scripts/gpu_ab.sh: ARMS, CFGS, ROUNDS) on the same box.  A test failure
# (pytest exit 1) still runs the A/B; any other exit status ends the script.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-tab}; mkdir -p $OUT
if [ -n "${TESTS:-}" ]; then
  timeout -k 10 ${TEST_TIMEOUT:-700} python -u -m pytest $TESTS -x -v --timeout 150 --timeout-method thread > $OUT/tests.log 2>&1
  rc=$?; tail -3 $OUT/tests.log
  [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
fi
[ -z "${ARMS:-}" ] || TAG=${TAG:-tab} bash scripts/gpu_ab.sh
