# predict-pass timing per library arm (KM_LIB), alternating, one box:
#   ARMS="libkmeans_amd.so libkmeans_amd_abl1.so" CFG=c3 TAG=r5_abl bash scripts/gpu_predict_ab.sh
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
P=assignment--2-group7-distributed-k-means_amd
OUT=gpurun_out/${TAG:-pab}; mkdir -p $OUT
for R in $(seq ${ROUNDS:-2}); do
  for A in ${ARMS:-libkmeans_amd.so}; do
    N=${A%.so}
    KM_LIB=$PWD/$P/$A timeout -k 10 300 python -u bench.py --config ${CFG:-c3} --steps ${STEPS:-2} --warmup 1 \
      --no-cpu-baseline --predict ${PRED:-10} > $OUT/$N.$R.json 2> $OUT/$N.$R.err || { echo "$A failed"; tail -5 $OUT/$N.$R.err; exit 1; }
    python3 -c "import json;d=json.load(open('$OUT/$N.$R.json'));p=d['predict'];print('$N $R', round(p['kernel_ms']['assign'],3), round(p['kernel_ms']['resolve'],3), round(p['ms_per_pass'],3), round(p['gb_s'],1))"
  done
done
