# bench every config on one GPU (short runs) to check paths and timings
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-cfg}; mkdir -p $OUT
for C in ${CFGS:-c2 c3 c5 c4}; do
  timeout -k 10 400 python -u bench.py --config $C --steps ${STEPS:-5} --warmup 2 --no-cpu-baseline > $OUT/$C.json 2> $OUT/$C.err || { echo "$C failed"; tail -5 $OUT/$C.err; exit 1; }
  python -c "import json;d=json.load(open('$OUT/$C.json'));print('$C', round(d['value'],3),'it/s', {k:round(v,3) for k,v in d['kernel_avg_ms'].items()}, d['resolve'], d['roofline']['bound'], round(d['roofline']['achieved'],1), round(d['roofline']['frac'],3))"
done
