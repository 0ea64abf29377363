# product library vs variants libkmeans_amd_<name>.so (make -C .../csrc alt
# ALT_FLAGS=... ALT_OUT=../libkmeans_amd_<name>.so), alternating runs on one
# box; optional parity subset of the product (or PLIB variant) first:
#   TESTS="one_step or near_ties" CFGS="c5 c4" ALTS="alt alt2" bash scripts/gpu_altab.sh
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
P=assignment--2-group7-distributed-k-means_amd
OUT=gpurun_out/${TAG:-altab}; mkdir -p $OUT
cp $P/libkmeans_amd.so $OUT/prod.so
if [ -n "${PLIB:-}" ]; then cp $P/libkmeans_amd_$PLIB.so $P/libkmeans_amd.so; fi
if [ -n "${TESTS:-}" ]; then
  timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "$TESTS" > $OUT/tests.log 2>&1 || { echo "tests failed"; tail -30 $OUT/tests.log; cp $OUT/prod.so $P/libkmeans_amd.so; exit 1; }
  tail -2 $OUT/tests.log
fi
for CFG in ${CFGS:-c5}; do
  for V in prod ${ALTS:-alt} prod ${ALTS:-alt}; do
    if [ $V = prod ]; then cp $OUT/prod.so $P/libkmeans_amd.so; else cp $P/libkmeans_amd_$V.so $P/libkmeans_amd.so; fi
    timeout -k 10 300 python -u bench.py --config $CFG --steps ${STEPS:-10} --warmup 2 --no-cpu-baseline > $OUT/$CFG.$V.json 2> $OUT/$CFG.$V.err || { echo "$CFG $V failed"; tail -5 $OUT/$CFG.$V.err; cp $OUT/prod.so $P/libkmeans_amd.so; exit 1; }
    python3 -c "import json;d=json.load(open('$OUT/$CFG.$V.json'));print('$CFG $V', round(d['value'],2), round(d['ms_per_step'],3), {k:round(v,3) for k,v in d['kernel_avg_ms'].items()})"
  done
done
cp $OUT/prod.so $P/libkmeans_amd.so
