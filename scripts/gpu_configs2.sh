# other configs on one GPU: c4 (1B x 32, k=1024), c3_shard8, the wide-row config
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-cfg2}; mkdir -p $OUT
for spec in "c3_shard8 20 3" "w784 5 2" "c4 3 1"; do
  set -- $spec
  timeout -k 10 400 python -u bench.py --config $1 --steps $2 --warmup $3 --no-cpu-baseline > $OUT/$1.json 2> $OUT/$1.err || { tail -5 $OUT/$1.err; exit 1; }
  python3 -c "import json;d=json.load(open('$OUT/$1.json'));print('$1', round(d['value'],3), round(d['ms_per_step'],3), round(d['roofline']['frac'],3), d['roofline']['kernel'], {k:round(v,3) for k,v in d['kernel_avg_ms'].items()}, d['resolve'])"
done
