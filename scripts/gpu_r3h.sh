# 16-wave k_assign_mfma for dp <= 64: GPU suite + smoke, then the rocprofv3
# kernel trace of the c4 bench line (compute_sse=True, its BASELINE config)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r3h}; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { echo tests failed; grep -E "FAILED|Error" $OUT/gpu_tests.log | head; tail -30 $OUT/gpu_tests.log; exit 1; }
tail -1 $OUT/gpu_tests.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo smoke failed; tail -20 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
for C in c4; do
  timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/$C -o run -- python3 bench.py --config $C --steps 6 --warmup 2 --no-cpu-baseline > $OUT/$C.json 2> $OUT/$C.err || { echo "$C prof failed"; tail -5 $OUT/$C.err; exit 1; }
  python3 scripts/trace_summary.py $OUT/$C/run_kernel_trace.csv --json $OUT/$C.summary.json > $OUT/$C.summary.txt && head -6 $OUT/$C.summary.txt
  python3 -c "import json;d=json.load(open('$OUT/$C.json'));print('$C', round(d['value'],3), round(d['ms_per_step'],3), {k:round(v,3) for k,v in d['kernel_avg_ms'].items()}, d['roofline']['frac'])"
done
