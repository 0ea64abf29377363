# A/B of an env knob on the c3 bench (after the GPU parity tests):
#   VAR=KM_DEFER VALS="0 1" bash scripts/gpu_ab.sh
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${TAG:-ab}
if [ "${SKIP_TESTS:-0}" != 1 ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/${TAG}_tests.log
  [ $rc -ne 0 ] && exit 1
fi
for V in ${VALS}; do
  env $VAR=$V timeout -k 10 300 python -u bench.py --config ${CFG:-c3} --steps ${STEPS:-10} --warmup 2 --no-cpu-baseline > gpurun_out/${TAG}_$V.json 2> gpurun_out/${TAG}_$V.err || { tail -5 gpurun_out/${TAG}_$V.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/${TAG}_$V.json'));print('$VAR=$V', round(d['value'],2),'it/s', {k:round(v,3) for k,v in d['kernel_avg_ms'].items()}, d['resolve'], round(d['roofline']['frac'],3))"
done
