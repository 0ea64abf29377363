# fused-kernel ablations only (KM_ABLATE list), c3 bench, kernel avg ms
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-abl}; mkdir -p $OUT
for A in ${ABL_LIST:-0}; do
  KM_ABLATE=$A timeout -k 10 300 python -u bench.py --config ${CFG:-c3} --steps 5 --warmup 1 --no-cpu-baseline > $OUT/abl$A.json 2> $OUT/abl$A.err || { echo "abl $A failed"; tail -5 $OUT/abl$A.err; exit 1; }
  python -c "import json;d=json.load(open('$OUT/abl$A.json'));print('ABL=$A', round(d['value'],2),'it/s', {k:round(v,3) for k,v in d['kernel_avg_ms'].items()})"
  grep "km stamps" $OUT/abl$A.err | tail -2 || true
done
