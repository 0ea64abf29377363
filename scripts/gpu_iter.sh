# quick correctness + perf iteration: parity tests, then bench variants
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${TAG:-iter}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -5 gpurun_out/${TAG}_tests.log
[ $rc -ne 0 ] && exit 1
for F in ${FUSED_LIST:-1 0}; do
  KM_FUSED=$F timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/${TAG}_bench_f$F.json 2> gpurun_out/${TAG}_bench_f$F.err || { tail -5 gpurun_out/${TAG}_bench_f$F.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/${TAG}_bench_f$F.json'));print('fused=$F', round(d['value'],2),'it/s', {k:round(v,3) for k,v in d['kernel_avg_ms'].items()}, d['resolve'], round(d['roofline']['frac'],3))"
done
