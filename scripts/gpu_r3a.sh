# round-3 baseline: rocprofv3 kernel trace of the c5 poor-seed bench (split of
# the statistics time over k_hist / k_scatter / k_segsum) and the c3 bench
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r3a}; mkdir -p $OUT
for C in ${CFGS:-c5_poor}; do
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/$C -o run -- python3 bench.py --config $C --steps ${STEPS:-4} --warmup 1 --no-cpu-baseline > $OUT/$C.json 2> $OUT/$C.err || { echo "$C failed"; tail -5 $OUT/$C.err; exit 1; }
  python3 scripts/trace_summary.py $OUT/$C/run_kernel_trace.csv > $OUT/$C.summary.txt && cat $OUT/$C.summary.txt
done
for C in ${BENCH:-c3}; do
  timeout -k 10 300 python -u bench.py --config $C --steps 20 --warmup 3 --no-cpu-baseline > $OUT/bench_$C.json 2> $OUT/bench_$C.err || { echo "bench $C failed"; tail -5 $OUT/bench_$C.err; exit 1; }
  python3 -c "import json;d=json.load(open('$OUT/bench_$C.json'));print('$C', round(d['value'],3), round(d['ms_per_step'],3), {k:round(v,3) for k,v in d['kernel_avg_ms'].items()}, d['roofline']['frac'])"
done
