#!/bin/bash
# full -m gpu suite, then the c3 bench line (default flags) and its rocprofv3
# kernel-stats run, then the c2 line
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/r2b; mkdir -p $OUT
timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1
rc=$?
tail -3 $OUT/gpu_tests.log; grep -E "FAILED|ERROR" $OUT/gpu_tests.log | head
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print(\"smoke ok\")" > $OUT/smoke.log 2>&1 || { tail -5 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
timeout -k 10 400 python3 bench.py > $OUT/bench_c3.json 2> $OUT/bench_c3.err || exit $?
cat $OUT/bench_c3.json
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_c3 -o run -- python3 bench.py --no-cpu-baseline > $OUT/prof_c3.log 2>&1 || exit $?
timeout -k 10 300 python3 bench.py --config c2 --steps 200 --warmup 20 --no-cpu-baseline > $OUT/bench_c2.json 2> $OUT/bench_c2.err || exit $?
cat $OUT/bench_c2.json
exit $rc
