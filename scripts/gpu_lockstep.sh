# lockstep full-scan chunk pass: the product (pairs decided per entry) on the
# parity tests that reach k_fullscan, timing at c3 / c5, then the pair-skip
# variant (libkmeans_amd_pairskip.so: a pair skipped when its first entry is
# resolved) on the same tests -- expected to fail
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
P=assignment--2-group7-distributed-k-means_amd
OUT=gpurun_out/lockstep; mkdir -p $OUT
SEL="near_ties or triple or one_step or randn or candidate or c5_shape or tight or golden"
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_contraction.py -x -q --timeout 200 --timeout-method thread -k "$SEL" > $OUT/product.log 2>&1 || { echo product failed; grep -E "FAILED|Error" $OUT/product.log | head; tail -20 $OUT/product.log; exit 1; }
tail -1 $OUT/product.log
for C in c3 c5; do
  timeout -k 10 300 python -u bench.py --config $C --steps 10 --warmup 2 --no-cpu-baseline > $OUT/bench_$C.json 2> $OUT/bench_$C.err || { echo "bench $C failed"; tail -5 $OUT/bench_$C.err; exit 1; }
  python3 -c "import json;d=json.load(open('$OUT/bench_$C.json'));print('$C', round(d['value'],3), {k:round(v,3) for k,v in d['kernel_avg_ms'].items()}, d['resolve'])"
done
cp $P/libkmeans_amd.so $OUT/prod.so
cp $P/libkmeans_amd_pairskip.so $P/libkmeans_amd.so
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_contraction.py -q --timeout 200 --timeout-method thread -k "$SEL" > $OUT/pairskip.log 2>&1
echo "pairskip rc=$?"; grep -E "^FAILED|passed|failed" $OUT/pairskip.log | tail -25
cp $OUT/prod.so $P/libkmeans_amd.so
