# A/B/A of two builds of the library on one box: libkmeans_amd_prev.so vs
# libkmeans_amd_new.so copied over the product name between bench runs
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
P=assignment--2-group7-distributed-k-means_amd
for V in new prev new prev; do
  cp $P/libkmeans_amd_$V.so $P/libkmeans_amd.so
  timeout -k 10 300 python -u bench.py --config ${CFG:-c3} --steps ${STEPS:-20} --warmup 3 --no-cpu-baseline > gpurun_out/ab_$V.json 2> gpurun_out/ab_$V.err || { tail -5 gpurun_out/ab_$V.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/ab_$V.json'));print('$V', round(d['value'],2), {k:round(v,3) for k,v in d['kernel_avg_ms'].items()})"
done
cp $P/libkmeans_amd_new.so $P/libkmeans_amd.so
