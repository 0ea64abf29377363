# A/B of library builds on one box, alternating runs (never ranks builds across
# boxes: MI355X_MICROARCH.md 'DVFS give-back' item 5).  Each arm is a library
# file under the package directory, selected per process through KM_LIB
# (nothing is copied over the product library):
#   ARMS="libkmeans_amd.so libkmeans_amd_f32.so" CFGS="c3 c5" TAG=r4_shape bash scripts/gpu_ab.sh
# optional: ROUNDS (default 2), STEPS (default 20), WARMUP (default 3), SSE (bench --sse)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
P=assignment--2-group7-distributed-k-means_amd
OUT=gpurun_out/${TAG:-ab}; mkdir -p $OUT
EXTRA=""
if [ -n "${SSE:-}" ]; then EXTRA="--sse $SSE"; fi
for CFG in ${CFGS:-c3}; do
  for R in $(seq ${ROUNDS:-2}); do
    for A in ${ARMS:-libkmeans_amd.so}; do
      N=${A%.so}
      KM_LIB=$PWD/$P/$A timeout -k 10 400 python -u bench.py --config $CFG --steps ${STEPS:-20} --warmup ${WARMUP:-3} \
        --no-cpu-baseline $EXTRA > $OUT/$CFG.$N.$R.json 2> $OUT/$CFG.$N.$R.err || { echo "$CFG $A failed"; tail -5 $OUT/$CFG.$N.$R.err; exit 1; }
      python3 -c "import json;d=json.load(open('$OUT/$CFG.$N.$R.json'));print('$CFG $N $R', round(d['value'],3), round(d['ms_per_step'],3), {k:round(v,3) for k,v in d['kernel_avg_ms'].items()}, d['resolve'])"
    done
  done
done
