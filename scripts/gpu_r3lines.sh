# bench lines (no CPU baseline) for the large configs: c5, c5_poor, c4, c3_shard8
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r3lines}; mkdir -p $OUT
for C in ${CFGS:-c5 c5_poor c4 c3_shard8}; do
  timeout -k 10 300 python -u bench.py --config $C --steps 10 --warmup 2 --no-cpu-baseline > $OUT/$C.json 2> $OUT/$C.err || { echo "$C failed"; tail -5 $OUT/$C.err; exit 1; }
  python3 -c "import json;d=json.load(open('$OUT/$C.json'));print('$C', round(d['value'],3), round(d['ms_per_step'],3), {k:round(v,3) for k,v in d['kernel_avg_ms'].items()}, round(d['roofline']['frac'],4), d['roofline']['traffic'])"
done
