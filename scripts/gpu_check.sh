# HEAD check: GPU parity tests, smoke, default bench, fused-kernel ablations
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-check}; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { echo tests failed; tail -20 $OUT/gpu_tests.log; exit 1; }
tail -2 $OUT/gpu_tests.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo smoke failed; tail -20 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
timeout -k 10 600 python -u bench.py --steps 10 --warmup 2 --cpu-seconds 5 > $OUT/bench.json 2> $OUT/bench.err || { echo bench failed; tail -20 $OUT/bench.err; exit 1; }
cat $OUT/bench.json
for A in ${ABL_LIST:-}; do
  KM_ABLATE=$A timeout -k 10 300 python -u bench.py --steps 5 --warmup 1 --no-cpu-baseline > $OUT/abl$A.json 2> $OUT/abl$A.err || { echo "abl $A failed"; tail -5 $OUT/abl$A.err; exit 1; }
  python -c "import json;d=json.load(open('$OUT/abl$A.json'));print('ABL=$A', round(d['value'],2),'it/s', {k:round(v,3) for k,v in d['kernel_avg_ms'].items()})"
done
