# A/B of several builds of the library on one box, interleaved:
#   LIBS="cur fused" CFGS="c3 c2" ROUNDS=2 bash scripts/gpu_abn.sh
# (libkmeans_amd_<name>.so copied over the product name between bench runs)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
P=assignment--2-group7-distributed-k-means_amd
OUT=gpurun_out/${TAG:-abn}; mkdir -p $OUT
cp $P/libkmeans_amd.so $OUT/orig.so
for R in $(seq ${ROUNDS:-2}); do
  for C in ${CFGS:-c3}; do
    for V in ${LIBS}; do
      cp $P/libkmeans_amd_$V.so $P/libkmeans_amd.so
      timeout -k 10 300 python -u bench.py --config $C --steps ${STEPS:-20} --warmup 3 --no-cpu-baseline ${BARGS:-} > $OUT/${C}_${V}_$R.json 2> $OUT/${C}_${V}_$R.err || { tail -5 $OUT/${C}_${V}_$R.err; cp $OUT/orig.so $P/libkmeans_amd.so; exit 1; }
      python3 -c "import json;d=json.load(open('$OUT/${C}_${V}_$R.json'));print('$C $V $R', round(d['value'],2), round(d['ms_per_step'],3), {k:round(v,3) for k,v in d['kernel_avg_ms'].items()}, d['resolve'])"
    done
  done
done
cp $OUT/orig.so $P/libkmeans_amd.so
