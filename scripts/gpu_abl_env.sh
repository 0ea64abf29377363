# Diagnostic-library ablations A/B on one box (results wrong by design; wall
# time of the assign kernel from HIP events): ENVS="KM_ABLATE=11 KM_ABLATE=15"
# CFG=c5 TAG=... bash scripts/gpu_abl_env.sh
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
P=assignment--2-group7-distributed-k-means_amd
OUT=gpurun_out/${TAG:-ablenv}; mkdir -p $OUT
for R in $(seq ${ROUNDS:-2}); do
  for E in $ENVS; do
    N=${E//=/_}
    env KM_LIB=$PWD/$P/libkmeans_amd_diag.so $E timeout -k 10 400 python -u bench.py --config ${CFG:-c5} --steps ${STEPS:-5} \
      --warmup ${WARMUP:-2} --no-cpu-baseline > $OUT/$N.$R.json 2> $OUT/$N.$R.err || { echo "$E failed"; tail -5 $OUT/$N.$R.err; exit 1; }
    python3 -c "import json;d=json.load(open('$OUT/$N.$R.json'));print('$E $R', d['steps_ran'], {k:round(v,3) for k,v in d['kernel_avg_ms'].items()})"
  done
done
