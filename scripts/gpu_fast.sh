#!/bin/bash
# fast-screen round: parity tests of every screen, then c3 bench per screen
cd "${GRAFT_REPO_ROOT:-/root/repo}"
out=gpurun_out/fast
mkdir -p $out
if [ -z "$SKIP_TESTS" ]; then timeout -k 10 900 python -u -m pytest -v --timeout 300 --timeout-method thread tests/test_gpu_fast_screen.py > $out/tests.log 2>&1
rc=$?; else rc=0; fi
echo "tests rc=$rc"
tail -3 $out/tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
for m in ${SCREENS:-2 3 0}; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --screen $m > $out/bench_s$m.json 2> $out/bench_s$m.err || exit $?
  cat $out/bench_s$m.json
done
