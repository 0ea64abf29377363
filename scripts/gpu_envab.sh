# runs of the diagnostic library under several environment settings, one box:
#   RUNS="KM_FUSED=0,KM_TOP2=1 KM_FUSED=1" CFG=c3 bash scripts/gpu_envab.sh
# (each run: comma-separated VAR=VALUE list; the product library is restored)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
P=assignment--2-group7-distributed-k-means_amd
OUT=gpurun_out/${TAG:-envab}; mkdir -p $OUT
cp $P/libkmeans_amd.so $OUT/prod.so
cp $P/libkmeans_amd_diag.so $P/libkmeans_amd.so
i=0
for RUN in ${RUNS}; do
  i=$((i+1))
  ENVS=$(echo $RUN | tr ',' ' ')
  env $ENVS timeout -k 10 300 python -u bench.py --config ${CFG:-c3} --steps ${STEPS:-10} --warmup 2 --no-cpu-baseline ${BARGS:-} > $OUT/r$i.json 2> $OUT/r$i.err || { echo "$RUN failed"; tail -5 $OUT/r$i.err; cp $OUT/prod.so $P/libkmeans_amd.so; exit 1; }
  python3 -c "import json;d=json.load(open('$OUT/r$i.json'));print('$RUN', round(d['value'],2), round(d['ms_per_step'],3), {k:round(v,3) for k,v in d['kernel_avg_ms'].items()}, d['resolve'])"
done
cp $OUT/prod.so $P/libkmeans_amd.so
