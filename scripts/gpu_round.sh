# Round artefacts on one box: GPU parity suite, smoke, default bench (with the
# CPU baseline), rocprofv3 kernel trace of the same bench (summary with gated
# no-ops dropped, scripts/trace_summary.py).  TAG names the output directory.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-round}; mkdir -p $OUT
if [ -z "${SKIP_TESTS:-}" ]; then
  timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { echo tests failed; tail -20 $OUT/gpu_tests.log; exit 1; }
  tail -1 $OUT/gpu_tests.log
  timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo smoke failed; tail -20 $OUT/smoke.log; exit 1; }
  tail -1 $OUT/smoke.log
fi
for CFG in ${CFGS:-c3}; do
  timeout -k 10 500 python -u bench.py --config $CFG ${BENCH_ARGS:-} > $OUT/bench_$CFG.json 2> $OUT/bench_$CFG.err || { echo bench $CFG failed; tail -20 $OUT/bench_$CFG.err; exit 1; }
  cat $OUT/bench_$CFG.json
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace_$CFG -o run -- python3 bench.py --config $CFG --no-cpu-baseline ${BENCH_ARGS:-} > $OUT/trace_bench_$CFG.json 2> $OUT/trace_$CFG.err || { echo trace $CFG failed; tail -5 $OUT/trace_$CFG.err; exit 1; }
  python3 scripts/trace_summary.py $(ls $OUT/trace_$CFG/*kernel_trace.csv | head -1) > $OUT/trace_summary_$CFG.txt && head -8 $OUT/trace_summary_$CFG.txt
done
