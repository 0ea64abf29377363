# round-3 validation: GPU parity suite + smoke, then rocprofv3 kernel traces
# (no-op dispatches filtered by scripts/trace_summary.py) of the benches in CFGS
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r3b}; mkdir -p $OUT
if [ "${SKIP_TESTS:-0}" != 1 ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > $OUT/gpu_tests.log 2>&1 || { echo tests failed; grep -E "FAILED|Error|error" $OUT/gpu_tests.log | head -20; tail -30 $OUT/gpu_tests.log; exit 1; }
  tail -2 $OUT/gpu_tests.log
  timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo smoke failed; tail -20 $OUT/smoke.log; exit 1; }
  tail -1 $OUT/smoke.log
fi
for C in ${CFGS:-}; do
  timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/$C -o run -- python3 bench.py --config $C --steps ${STEPS:-6} --warmup ${WARM:-2} --no-cpu-baseline > $OUT/$C.json 2> $OUT/$C.err || { echo "$C failed"; tail -5 $OUT/$C.err; exit 1; }
  python3 scripts/trace_summary.py $OUT/$C/run_kernel_trace.csv --json $OUT/$C.summary.json > $OUT/$C.summary.txt && head -12 $OUT/$C.summary.txt
  python3 -c "import json;d=json.load(open('$OUT/$C.json'));print('$C', round(d['value'],3), round(d['ms_per_step'],3), d['steps_ran'], {k:round(v,3) for k,v in d['kernel_avg_ms'].items()}, round(d['roofline']['frac'],4))"
done
for C in ${BENCH:-}; do
  timeout -k 10 300 python -u bench.py --config $C --steps ${BSTEPS:-20} --warmup 3 --no-cpu-baseline > $OUT/bench_$C.json 2> $OUT/bench_$C.err || { echo "bench $C failed"; tail -5 $OUT/bench_$C.err; exit 1; }
  python3 -c "import json;d=json.load(open('$OUT/bench_$C.json'));print('$C', round(d['value'],3), round(d['ms_per_step'],3), d['steps_ran'], {k:round(v,3) for k,v in d['kernel_avg_ms'].items()}, round(d['roofline']['frac'],4))"
done
