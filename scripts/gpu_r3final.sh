# round-3 close: GPU suite + smoke, the default bench line (c3, with the CPU
# baseline), rocprofv3 kernel trace of c3, and the c2 / c3_shard8 / w784 lines
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r3final}; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { echo tests failed; grep -E "FAILED|Error" $OUT/gpu_tests.log | head; tail -30 $OUT/gpu_tests.log; exit 1; }
tail -1 $OUT/gpu_tests.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo smoke failed; tail -20 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
timeout -k 10 400 python -u bench.py > $OUT/bench_default.json 2> $OUT/bench_default.err || { echo bench failed; tail -5 $OUT/bench_default.err; exit 1; }
cat $OUT/bench_default.json
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/c3 -o run -- python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline > $OUT/c3.json 2> $OUT/c3.err || { echo c3 prof failed; tail -5 $OUT/c3.err; exit 1; }
python3 scripts/trace_summary.py $OUT/c3/run_kernel_trace.csv --json $OUT/c3.summary.json > $OUT/c3.summary.txt && head -6 $OUT/c3.summary.txt
for C in c2 c3_shard8 w784; do
  timeout -k 10 300 python -u bench.py --config $C --steps 30 --warmup 5 --no-cpu-baseline > $OUT/bench_$C.json 2> $OUT/bench_$C.err || { echo "bench $C failed"; tail -5 $OUT/bench_$C.err; exit 1; }
  python3 -c "import json;d=json.load(open('$OUT/bench_$C.json'));print('$C', round(d['value'],2), round(d['ms_per_step'],4), {k:round(v,4) for k,v in d['kernel_avg_ms'].items()}, d['roofline']['frac'], d['roofline']['traffic'])"
done
