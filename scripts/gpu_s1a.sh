# Round-5 development runs on one box: the given GPU test files, then the c3
# bench (no CPU leg).  TAG names gpurun_out/<TAG>; TESTS the test files.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-s1a}; mkdir -p $OUT
timeout -k 10 700 python -u -m pytest ${TESTS:-tests/test_gpu_s1.py} -v --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?
echo "pytest rc=$rc"; grep -E "PASS|FAIL|ERROR|passed|failed" $OUT/tests.log | tail -40
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
for CFG in ${CFGS:-c3}; do
  timeout -k 10 300 python -u bench.py --config $CFG --steps ${STEPS:-20} --no-cpu-baseline ${BENCH_ARGS:-} > $OUT/bench_$CFG.json 2> $OUT/bench_$CFG.err
  rc=$?; echo "bench $CFG rc=$rc"; cat $OUT/bench_$CFG.json; tail -3 $OUT/bench_$CFG.err
  if [ $rc -ne 0 ]; then exit $rc; fi
done
